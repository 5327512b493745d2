#!/bin/bash
# Round 6: wave-strided long-line / chain-vertex loops with four loads in
# flight (big path) -- big-path and UC GPU parity tests, F4 and UC lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "c1000 or big_teams or uc_ or sslp or c100" > $O/pytest_unroll.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_unroll.log | tail -24
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --tol-run 0 --no-cpu-baseline --only f4 --hbm-steps 5 > $O/f4_unroll.json 2> $O/f4_unroll.log || { echo "f4 failed"; tail -20 $O/f4_unroll.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/f4_unroll.json'))['f4'];print('F4', d['ms_per_step'], d['iter0_s'], d['roofline'].get('polish_ms'), d['roofline'].get('kernel_ms'), d.get('ef_bracket',{}).get('ok'))"
timeout -k 10 300 python3 -u tools/mid_phase_probe.py farmer1000 1000 5 3 > $O/f4_phases_unroll.txt 2>&1 || { echo "phase probe failed"; tail -20 $O/f4_phases_unroll.txt; exit 1; }
grep -v amdgpu.ids $O/f4_phases_unroll.txt | cut -c1-300
timeout -k 10 600 python3 -u bench.py --tol-run 0 --no-cpu-baseline --only uc > $O/uc_unroll.json 2> $O/uc_unroll.log || { echo "uc failed"; tail -20 $O/uc_unroll.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/uc_unroll.json'))['uc'];print('UC', {k: d[k] for k in ('iter0_s','ms_per_ph_iteration','trivial_bound','lagrangian_bound','not_optimal_after','wall_s')})"
echo ALLDONE
