#!/bin/bash
# mid-size polish exit reasons at F3 iterations 6..10 against the KKT regularisation
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for d in ${DELTAS:-1e-5 1e-9 1e-11}; do
  PHGPU_KKT_DELTA=$d timeout -k 10 250 python -u tools/mid_polish_prof.py 10000 100 6 4 > gpurun_out/delta_$d.txt 2>&1 || { echo "delta $d failed"; tail -5 gpurun_out/delta_$d.txt; exit 1; }
  echo "== delta $d"; grep -v -e Warn -e amdgpu.ids gpurun_out/delta_$d.txt
done
