#!/bin/bash
# Round 6 measurement pass (from gpu_r05_prof.sh) (one GPU call): the F2 line (fused pass) as in round 4:
#  1. FETCH_SIZE / WRITE_SIZE calibration on known byte counts for the access
#     patterns of the kernels (tools/fetch_calib.hip);
#  2. every companion workload profiled ON ITS OWN through `bench.py --only`,
#     so the PMC window (the last --hbm-steps solve calls) is the exact window
#     the bench line's HIP events time; F4 also on its Iter0 (the streaming
#     PDHG regime);
#  3. the F2 headline profile as before.
# Usage: bash tools/gpu_r04_prof.sh [TAG] ["calib f3 sslp f4 f2"]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
TAG=${1:-r06}
SEL=${2:-"f2"}
on() { [[ " $SEL " == *" $1 "* ]]; }
mkdir -p $O $R/profiles/$TAG
cd $R
export TMPDIR=/tmp
if on calib; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/calib_fetch -o run -- ./tools/fetch_calib > $O/calib.log 2>&1 || { echo "calib fetch failed"; tail -20 $O/calib.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/calib_write -o run -- ./tools/fetch_calib >> $O/calib.log 2>&1 || { echo "calib write failed"; tail -20 $O/calib.log; exit 1; }
  python3 tools/fetch_calib_summary.py $O/calib_fetch $O/calib_write $O/calib.log > $O/fetch_calibration.json || { echo "calib summary failed"; exit 1; }
  cp $O/fetch_calibration.json profiles/$TAG/
  cat $O/fetch_calibration.json
fi
prof() {  # name, window, workload tag, bench args...
  local N=$1 W=$2 WL=$3; shift 3
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${N}_stats -o run -- python3 bench.py "$@" > $O/${N}_stats.json 2> $O/${N}_stats.log || { echo "rocprof $N stats failed"; tail -30 $O/${N}_stats.log; return 1; }
  timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${N}_fetch -o run -- python3 bench.py "$@" > $O/${N}_fetch.log 2>&1 || { echo "pmc $N fetch failed"; tail -30 $O/${N}_fetch.log; return 1; }
  timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${N}_write -o run -- python3 bench.py "$@" > $O/${N}_write.log 2>&1 || { echo "pmc $N write failed"; tail -30 $O/${N}_write.log; return 1; }
  python3 tools/pmc_summary.py $O/${N}_fetch $O/${N}_write $O/${N}_stats $O/pmc_summary_$N.json $WL $W > /dev/null || { echo "pmc $N summary failed"; return 1; }
  cp $O/pmc_summary_$N.json profiles/$TAG/pmc_summary_$N.json
  cp $O/${N}_stats.json profiles/$TAG/${N}_line_under_rocprof.json
  cp $(find $O/${N}_stats -name '*kernel_stats.csv' | head -1) profiles/$TAG/${N}_kernel_stats.csv
  echo "profiled $N"
}
NOCPU="--tol-run 0 --no-cpu-baseline"
on f3 && { prof f3 5 farmer10k_c100 $NOCPU --only f3 --hbm-steps 5 --warmup 5 || exit 1; }
on sslp && { prof sslp 5 sslp10k $NOCPU --only sslp --hbm-steps 5 --warmup 5 || exit 1; }
if on f4; then
  prof f4 5 farmer1k_c1000 $NOCPU --only f4 --hbm-steps 5 --f4-bracket 0 || exit 1
  python3 tools/pmc_summary.py $O/f4_fetch $O/f4_write $O/f4_stats $O/pmc_summary_f4_iter0.json farmer1k_c1000 first > /dev/null || { echo "pmc f4 iter0 summary failed"; exit 1; }
  cp $O/pmc_summary_f4_iter0.json profiles/$TAG/
fi
on f2 && { prof f2 20 farmer10k_c1 $NOCPU --hbm-crops 0 --sslp-scens 0 --f4-scens 0 --uc-scens 0 || exit 1; }
echo ALLDONE
