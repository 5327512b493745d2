#!/bin/bash
# F3 graph repro, then F3 ms per PH iteration and polish phases at refinement tolerances
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/repro_f3.py 10000 100 1 3 > gpurun_out/repro_f3.log 2>&1 || { echo "F3 repro FAILED"; grep -v "^frame" gpurun_out/repro_f3.log | tail -6; exit 1; }
echo "F3 repro ok"
for t in 1e-15 1e-13 1e-12; do
  PHGPU_KKT_REFINE_TOL=$t timeout -k 10 240 python -u tools/mid_polish_prof.py 10000 100 2 3 > gpurun_out/midprof_$t.log 2>&1 || { echo "midprof $t failed"; tail -5 gpurun_out/midprof_$t.log; exit 1; }
  echo "tol $t"; tail -3 gpurun_out/midprof_$t.log
done
