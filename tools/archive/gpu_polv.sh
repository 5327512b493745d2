#!/bin/bash
# One GPU call: the GPU parity suite, then the mid-size polish phase clocks
# at F3 (farmer c=100, 10k scenarios, PH iterations 30-33).
# Usage: bash tools/gpu_polv.sh TAG   (outputs under gpurun_out/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
T=${1:-x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 || { tail -40 gpurun_out/pytest_$T.log; exit 1; }
tail -3 gpurun_out/pytest_$T.log
timeout -k 10 300 python -u tools/mid_polish_prof.py 10000 100 30 4 > gpurun_out/midprof_$T.log 2>&1 || { tail -20 gpurun_out/midprof_$T.log; exit 1; }
cat gpurun_out/midprof_$T.log
