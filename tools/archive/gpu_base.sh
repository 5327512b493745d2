#!/bin/bash
# One GPU call: the -m gpu parity suite, the F3 graph-replay repro (10k
# scenarios, c=100, graphs on, 3-iteration chunks), then the default bench line.
# Usage: bash tools/gpu_base.sh [tag]   (outputs under gpurun_out/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
TAG=${1:-base}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu_$TAG.log; exit 1; }
tail -3 $O/pytest_gpu_$TAG.log
timeout -k 10 300 python -u tools/repro_f3.py 10000 100 1 3 > $O/repro_f3_$TAG.log 2>&1 || { echo "repro failed"; tail -30 $O/repro_f3_$TAG.log; exit 1; }
tail -4 $O/repro_f3_$TAG.log
timeout -k 10 500 python -u bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo "bench failed"; tail -30 $O/bench_$TAG.err; exit 1; }
cat $O/bench_$TAG.json
echo ALLDONE
