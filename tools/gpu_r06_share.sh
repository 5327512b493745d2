#!/bin/bash
# Round 6: several big batches share the PDHG phase grid (big_team_grid) --
# the cylinder tests, then UC's cylinders line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "spin_the_wheel or async_spokes or uc_hub or big_teams" > $O/pytest_share.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_share.log | tail -8
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 -u bench.py --tol-run 0 --no-cpu-baseline --only uc > $O/uc_share.json 2> $O/uc_share.log || { echo "uc failed"; tail -20 $O/uc_share.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/uc_share.json'))['uc'];print('UC', {k: d[k] for k in ('iter0_s','ms_per_ph_iteration','trivial_bound','lagrangian_bound','best_outer_bound','not_optimal_after','wall_s')})"
echo ALLDONE
