#!/bin/bash
# Round 6: the mid-size polish's stored active sets (MidArgs::aset) -- the
# mid/big GPU parity tests, then polish clocks and bench lines of sslp / F3
# with the stored sets off (PHGPU_MID_ASET=0) and on, and F4 at HEAD
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "sslp or c100 or mid_path or c1000 or big_teams" > $O/pytest_aset.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_aset.log | tail -12
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
for a in 0 1; do
  PHGPU_MID_ASET=$a timeout -k 10 200 python3 -u tools/mid_polish_prof.py 10000 0 6 5 > $O/midprof_sslp_aset$a.txt 2>&1 || { echo "sslp prof $a failed"; tail $O/midprof_sslp_aset$a.txt; exit 1; }
  PHGPU_MID_ASET=$a timeout -k 10 200 python3 -u tools/mid_polish_prof.py 10000 100 30 5 > $O/midprof_f3_aset$a.txt 2>&1 || { echo "f3 prof $a failed"; tail $O/midprof_f3_aset$a.txt; exit 1; }
  echo "== aset $a"; grep -E "iters|polishes|per polish" $O/midprof_sslp_aset$a.txt $O/midprof_f3_aset$a.txt
done
for a in 0 1; do
  for w in sslp f3; do
    PHGPU_MID_ASET=$a timeout -k 10 300 python3 bench.py --tol-run 0 --no-cpu-baseline --only $w --hbm-steps 5 --warmup 5 > $O/${w}_aset$a.json 2> $O/${w}_aset$a.log || { echo "$w $a failed"; tail -20 $O/${w}_aset$a.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${w}_aset$a.json'))['$w'];print('$w ASET=$a', d['ms_per_step'], d['iter0_s'], d['pdhg_steps_per_solve'], d['pdhg_steps_max'])"
  done
done
timeout -k 10 300 python3 bench.py --tol-run 0 --no-cpu-baseline --only f4 --hbm-steps 5 > $O/f4_head.json 2> $O/f4_head.log || { echo "f4 failed"; tail -20 $O/f4_head.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/f4_head.json'))['f4'];print('F4', d['ms_per_step'], d['iter0_s'], d['roofline'].get('polish_ms'), d.get('ef_bracket',{}).get('ok'))"
echo ALLDONE
