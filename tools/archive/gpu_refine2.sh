#!/bin/bash
# mid-size polish (pinned rows) against the refinement stopping tolerance, F3 iterations 6..10
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for t in 1e-15 1e-13 1e-12 1e-11; do
  PHGPU_KKT_REFINE_TOL=$t timeout -k 10 250 python -u tools/mid_polish_prof.py 10000 100 6 4 > gpurun_out/ref_$t.txt 2>&1 || { echo "tol $t failed"; tail -5 gpurun_out/ref_$t.txt; exit 1; }
  echo "== tol $t"; grep -v -e Warn -e amdgpu.ids gpurun_out/ref_$t.txt
done
