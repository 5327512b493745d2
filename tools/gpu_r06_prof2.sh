#!/bin/bash
# Round 6: sslp with the 512- and 1024-thread mid-size geometries (A/B),
# then the F4 and F2 PMC profiles at HEAD (tools/gpu_r06_prof.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
for g in 512 1024; do
  PHGPU_MID_GEOM=$g timeout -k 10 300 python3 bench.py --tol-run 0 --no-cpu-baseline --only sslp --hbm-steps 5 --warmup 5 > $O/sslp_geom$g.json 2> $O/sslp_geom$g.log || { echo "sslp $g failed"; tail -20 $O/sslp_geom$g.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/sslp_geom$g.json'))['sslp'];print('GEOM=$g', d['ms_per_step'], d['iter0_s'], d['pdhg_steps_per_solve'], d['pdhg_steps_max'])"
done
bash tools/gpu_r06_prof.sh r06 "f4 f2" || exit 1
