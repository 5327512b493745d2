#!/bin/bash
# Round 6: smaller team caps on F4, and UC's cylinders line at two caps
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
f4() {
  local T=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --tol-run 0 --no-cpu-baseline --only f4 --hbm-steps 5 --f4-bracket 0 > $O/f4_$T.json 2> $O/f4_$T.log || { echo "f4 $T failed"; tail -20 $O/f4_$T.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/f4_$T.json'))['f4'];print('$T', d['ms_per_step'], d['iter0_s'], d['roofline'].get('polish_ms'), d['roofline'].get('kernel_ms'))"
}
f4 cap4 PHGPU_BIG_TEAM_CAP=4 || exit 1
f4 cap2 PHGPU_BIG_TEAM_CAP=2 || exit 1
uc() {
  local T=$1; shift
  env "$@" timeout -k 10 400 python3 -u bench.py --tol-run 0 --no-cpu-baseline --only uc > $O/uc_$T.json 2> $O/uc_$T.log || { echo "uc $T failed"; tail -20 $O/uc_$T.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/uc_$T.json'))['uc'];print('UC $T', {k: d[k] for k in ('iter0_s','ms_per_ph_iteration','lagrangian_bound','not_optimal_after','wall_s')})"
}
uc cap16 PHGPU_BIG_TEAM_CAP=16 || exit 1
uc cap4 PHGPU_BIG_TEAM_CAP=4 || exit 1
echo ALLDONE
