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
BARGS="--tol-run 0 --no-cpu-baseline --hbm-crops 0"
B3="--tol-run 0 --no-cpu-baseline --hbm-crops 0 --crops 100 --steps 5 --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- python3 bench.py $BARGS > $O/prof_stats.log 2>&1 || { echo "rocprof stats failed"; tail -30 $O/prof_stats.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- python3 bench.py $BARGS > $O/prof_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -30 $O/prof_fetch.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- python3 bench.py $BARGS > $O/prof_write.log 2>&1 || { echo "pmc write failed"; tail -30 $O/prof_write.log; exit 1; }
python3 tools/pmc_summary.py $O/prof_fetch $O/prof_write $O/prof_stats $O/pmc_summary.json 10000 1 20 > /dev/null || { echo "pmc summary failed"; exit 1; }
cp $O/pmc_summary.json profiles/$TAG/pmc_summary.json
# F3 companion (farmer c=100): the PDHG kernel's stats and HBM passes
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof3_stats -o run -- python3 bench.py $B3 > $O/prof3_stats.log 2>&1 || { echo "rocprof F3 stats failed"; tail -30 $O/prof3_stats.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof3_fetch -o run -- python3 bench.py $B3 > $O/prof3_fetch.log 2>&1 || { echo "pmc F3 fetch failed"; tail -30 $O/prof3_fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof3_write -o run -- python3 bench.py $B3 > $O/prof3_write.log 2>&1 || { echo "pmc F3 write failed"; tail -30 $O/prof3_write.log; exit 1; }
python3 tools/pmc_summary.py $O/prof3_fetch $O/prof3_write $O/prof3_stats $O/pmc_summary_c100.json 10000 100 5 > /dev/null || { echo "pmc F3 summary failed"; exit 1; }
cp $O/pmc_summary_c100.json profiles/$TAG/pmc_summary_c100.json
cp $O/prof3_stats/run_kernel_stats.csv profiles/$TAG/farmer10k_c100_kernel_stats.csv
cp $O/prof_stats/run_kernel_stats.csv profiles/$TAG/farmer10k_c1_kernel_stats.csv
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
cp $O/bench.json profiles/$TAG/bench_farmer10k_c1.json
echo ALLDONE
