#!/bin/bash
# Round 6: solves in the mid-size polish round's first pass (PHGPU_MID_SOLVES0
# 2 / 1) on F3 and sslp; the mid-path parity tests at 1; UC's cylinders line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
for v in 2 1; do
  for w in f3 sslp; do
    PHGPU_MID_SOLVES0=$v timeout -k 10 300 python3 bench.py --tol-run 0 --no-cpu-baseline --only $w --hbm-steps 5 --warmup 5 > $O/${w}_s0$v.json 2> $O/${w}_s0$v.log || { echo "$w $v failed"; tail -20 $O/${w}_s0$v.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${w}_s0$v.json'))['$w'];print('$w SOLVES0=$v', d['ms_per_step'], d['iter0_s'], d['pdhg_steps_per_solve'], d['pdhg_steps_max'], d.get('not_optimal_in_window'))"
  done
  PHGPU_MID_SOLVES0=$v timeout -k 10 200 python3 -u tools/mid_polish_prof.py 10000 100 30 5 > $O/midprof_f3_s0$v.txt 2>&1 || { echo "f3 prof $v failed"; exit 1; }
  grep -E "polishes|per polish" $O/midprof_f3_s0$v.txt
done
PHGPU_MID_SOLVES0=1 timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "sslp or c100 or mid_path" > $O/pytest_s01.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_s01.log | tail -8
timeout -k 10 400 python3 -u bench.py --tol-run 0 --no-cpu-baseline --only uc > $O/uc_long16.json 2> $O/uc_long16.log || { echo "uc failed"; tail -20 $O/uc_long16.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/uc_long16.json'))['uc'];print('UC', {k: d[k] for k in ('iter0_s','ms_per_ph_iteration','trivial_bound','lagrangian_bound','not_optimal_after','wall_s')})"
echo ALLDONE
