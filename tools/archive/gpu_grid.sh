#!/bin/bash
# F3 (Iter0 and steady state) with the phase kernels on the resident grid and on S blocks
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for g in 0 1; do
  PHGPU_MID_FULLGRID=$g timeout -k 10 300 python -u bench.py --steps 5 --warmup 5 --tol-run 0 --no-cpu-baseline > gpurun_out/grid_$g.json 2> gpurun_out/grid_$g.err || { echo "grid $g failed"; tail -20 gpurun_out/grid_$g.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/grid_$g.json'))['hbm_config'];print('fullgrid $g', d['ms_per_step'], d['iter0_s'], d['iter0_not_optimal'], d['roofline']['kernel_ms'], d['roofline']['launches_per_solve'])"
done
