#!/bin/bash
# One GPU call: the GPU parity suite, then the F2 line alone (no F3 / F4 /
# sslp / CPU baseline) -- the quick check of a one-wave path change.
# Usage: bash tools/gpu_f2.sh TAG   (outputs under gpurun_out/)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 || { tail -40 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
timeout -k 10 300 python -u bench.py --hbm-crops 0 --sslp-scens 0 --f4-scens 0 --no-cpu-baseline > gpurun_out/bench_f2_$T.json 2> gpurun_out/bench_f2_$T.err || { tail -20 gpurun_out/bench_f2_$T.err; exit 1; }
cat gpurun_out/bench_f2_$T.json
