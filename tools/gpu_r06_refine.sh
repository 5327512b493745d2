#!/bin/bash
# Round 6: polish A/B (refinement tolerance, then the KKT regularisation delta)
# PHGPU_REFINE_REL: min(tol, rel x 1e-9)) 1e-12 (default) / 1e-11 / 1e-10 on
# F4, F3 and sslp
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
run() {  # tag workload env...
  local T=$1 W=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --tol-run 0 --no-cpu-baseline --only $W --hbm-steps 5 --warmup 5 --f4-bracket 0 > $O/${W}_$T.json 2> $O/${W}_$T.log || { echo "$W $T failed"; tail -20 $O/${W}_$T.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/${W}_$T.json'))['$W'];r=d.get('roofline',{});print('$W $T', d['ms_per_step'], d['iter0_s'], d.get('pdhg_steps_per_solve'), d.get('pdhg_steps_max'), d.get('not_optimal_in_window'), r.get('polish_ms'))"
}
for cfg in "d7 PHGPU_X=0" "d8 PHGPU_KKT_DELTA=1e-8" "d9 PHGPU_KKT_DELTA=1e-9" "d6 PHGPU_KKT_DELTA=1e-6"; do
  set -- $cfg
  T=$1; shift
  run $T f4 "$@" || exit 1
  run $T f3 "$@" || exit 1
  run $T sslp "$@" || exit 1
done
echo ALLDONE
