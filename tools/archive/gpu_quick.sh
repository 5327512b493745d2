#!/bin/bash
# Quick GPU check: parity tests, then one short bench line (no CPU baseline).
# Usage: bash tools/gpu_quick.sh [extra bench args]   (outputs under gpurun_out/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/bench_quick.json 2> $O/bench_quick.err || { echo "bench failed"; tail -30 $O/bench_quick.err; exit 1; }
cat $O/bench_quick.json
