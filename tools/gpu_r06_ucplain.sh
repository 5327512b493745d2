#!/bin/bash
# Round 6: plain team launches when every live batch is big with a shared
# PDHG grid -- cylinder / team GPU tests, then UC's cylinders line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "spin_the_wheel or async_spokes or uc_hub or big_teams or c1000" > $O/pytest_ucplain.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_ucplain.log | tail -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 500 python3 -u bench.py --tol-run 0 --no-cpu-baseline --only uc > $O/uc_plain.json 2> $O/uc_plain.log || { echo "uc failed"; tail -20 $O/uc_plain.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/uc_plain.json'))['uc'];print('UC plain', {k: d[k] for k in ('iter0_s','ms_per_ph_iteration','trivial_bound','lagrangian_bound','best_outer_bound','not_optimal_after','wall_s')})"
echo ALLDONE
