#!/bin/bash
# mid-size polish with and without pinned rows: exit reasons at F3 iterations 6..10
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for v in 1 0; do
  PHGPU_MID_PIN=$v timeout -k 10 250 python -u tools/mid_polish_prof.py 10000 100 ${START:-6} 4 > gpurun_out/pin_$v.txt 2>&1 || { echo "pin $v failed"; tail -5 gpurun_out/pin_$v.txt; exit 1; }
  echo "== pin $v"; grep -v -e Warn -e amdgpu.ids gpurun_out/pin_$v.txt
done
