#!/bin/bash
# One GPU call: parity tests, rocprofv3 kernel stats + PMC HBM passes of the
# bench command, the per-kernel traffic summary, then the bench line.
# Usage: bash tools/gpu_full.sh [round-tag]   (outputs under gpurun_out/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
TAG=${1:-r01}
mkdir -p $O $R/profiles/$TAG
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
BARGS="--tol-run 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- python3 bench.py $BARGS > $O/prof_stats.log 2>&1 || { echo "rocprof stats failed"; tail -30 $O/prof_stats.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- python3 bench.py $BARGS > $O/prof_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -30 $O/prof_fetch.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- python3 bench.py $BARGS > $O/prof_write.log 2>&1 || { echo "pmc write failed"; tail -30 $O/prof_write.log; exit 1; }
python3 tools/pmc_summary.py $O/prof_fetch $O/prof_write $O/prof_stats $O/pmc_summary.json 10000 1 > /dev/null || { echo "pmc summary failed"; exit 1; }
cp $O/pmc_summary.json profiles/$TAG/pmc_summary.json
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
echo ALLDONE
