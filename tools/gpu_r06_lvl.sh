#!/bin/bash
# Round 6: level loops with their loads issued together (LDL' solve, big
# factor) and the big polish clocks compiled out -- mid/big parity tests,
# then F4 / F3 / sslp lines (twice, for the box's spread)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "sslp or c100 or mid_path or c1000 or big_teams" > $O/pytest_lvl.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_lvl.log | tail -8
[ $rc -eq 0 ] || exit 1
for k in 1 2; do
  for w in f4 f3 sslp; do
    timeout -k 10 300 python3 bench.py --tol-run 0 --no-cpu-baseline --only $w --hbm-steps 5 --warmup 5 --f4-bracket 0 > $O/${w}_lvl$k.json 2> $O/${w}_lvl$k.log || { echo "$w failed"; tail -20 $O/${w}_lvl$k.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${w}_lvl$k.json'))['$w'];r=d.get('roofline',{});print('$w', d['ms_per_step'], d['iter0_s'], d.get('pdhg_steps_per_solve'), d.get('pdhg_steps_max'), d.get('not_optimal_in_window'), r.get('polish_ms'))"
  done
done
echo ALLDONE
