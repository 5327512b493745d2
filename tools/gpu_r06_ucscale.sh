#!/bin/bash
# Round 6: UC cylinders (PH hub + Lagrangian spoke) at 16 and 64 scenarios
# (bench.py --only uc), statuses and time per PH iteration
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
for S in 16 64; do
  timeout -k 10 540 python3 -u bench.py --tol-run 0 --no-cpu-baseline --only uc --uc-scens $S > $O/uc_s$S.json 2> $O/uc_s$S.log || { echo "uc $S failed"; tail -5 $O/uc_s$S.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/uc_s$S.json'))['uc'];print('UC $S', {k: d[k] for k in ('iter0_s','ms_per_ph_iteration','trivial_bound','lagrangian_bound','best_outer_bound','not_optimal_after','wall_s')})"
done
echo ALLDONE
