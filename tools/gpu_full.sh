#!/bin/bash
# One GPU call: rocprofv3 kernel stats + PMC HBM passes of each bench
# workload ON ITS OWN (F2 headline, F3 c=100, sslp, F4 c=1000), the per-kernel traffic
# summaries (tools/pmc_summary.py refuses a window of another workload's
# kernels), then the default bench line.
# Usage: bash tools/gpu_full.sh [round-tag] ["f2 f3 sslp f4" | ... ] [bench]
#   (outputs under gpurun_out/; the default profiles all four, then benches)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
TAG=${1:-r03}
SEL=${2:-"f2 f3 sslp f4"}
BENCH=${3:-bench}
on() { [[ " $SEL " == *" $1 "* ]]; }
mkdir -p $O $R/profiles/$TAG
cd $R
export TMPDIR=/tmp
prof() {  # name, window, workload tag, bench args...
  local N=$1 W=$2 WL=$3; shift 3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${N}_stats -o run -- python3 bench.py "$@" > $O/${N}_stats.log 2>&1 || { echo "rocprof $N stats failed"; tail -30 $O/${N}_stats.log; return 1; }
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${N}_fetch -o run -- python3 bench.py "$@" > $O/${N}_fetch.log 2>&1 || { echo "pmc $N fetch failed"; tail -30 $O/${N}_fetch.log; return 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${N}_write -o run -- python3 bench.py "$@" > $O/${N}_write.log 2>&1 || { echo "pmc $N write failed"; tail -30 $O/${N}_write.log; return 1; }
  python3 tools/pmc_summary.py $O/${N}_fetch $O/${N}_write $O/${N}_stats $O/pmc_summary_$N.json $WL $W > /dev/null || { echo "pmc $N summary failed"; return 1; }
  cp $O/pmc_summary_$N.json profiles/$TAG/pmc_summary_$N.json
  cp $O/${N}_stats/run_kernel_stats.csv profiles/$TAG/${N}_kernel_stats.csv 2>/dev/null || cp $(find $O/${N}_stats -name '*kernel_stats.csv' | head -1) profiles/$TAG/${N}_kernel_stats.csv
}
ONE="--tol-run 0 --no-cpu-baseline --hbm-crops 0 --sslp-scens 0 --f4-scens 0"
on f2 && { prof f2 20 farmer10k_c1 $ONE || exit 1; }
on f3 && { prof f3 5 farmer10k_c100 $ONE --crops 100 --steps 5 --warmup 5 || exit 1; }
on sslp && { prof sslp 5 sslp10k --tol-run 0 --no-cpu-baseline --hbm-crops 0 --f4-scens 0 --scens 1000 --steps 5 --warmup 5 --sslp-scens 10000 || exit 1; }
on f4 && { prof f4 5 farmer1k_c1000 --tol-run 0 --no-cpu-baseline --hbm-crops 0 --sslp-scens 0 --scens 1000 --steps 5 --warmup 5 --f4-scens 1000 --hbm-steps 5 || exit 1; }
[ "$BENCH" = bench ] || { echo ALLDONE; exit 0; }
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
cp $O/bench.json profiles/$TAG/bench_farmer10k_c1.json
echo ALLDONE
