#!/bin/bash
# One GPU call: parity tests, bench line, rocprofv3 kernel stats, PMC HBM passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
BARGS="--steps 10 --warmup 3 --tol-run 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- python3 bench.py $BARGS > $O/prof_stats.log 2>&1 || { echo "rocprof stats failed"; tail -30 $O/prof_stats.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/prof_fetch -o run -- python3 bench.py $BARGS > $O/prof_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -30 $O/prof_fetch.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/prof_write -o run -- python3 bench.py $BARGS > $O/prof_write.log 2>&1 || { echo "pmc write failed"; tail -30 $O/prof_write.log; exit 1; }
echo ALLDONE
