#!/bin/bash
# F3 ms per PH iteration with the default mid-size geometry and with 512-thread blocks
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for g in 0 512; do
  PHGPU_MID_GEOM=$g timeout -k 10 300 python -u bench.py --crops 100 --steps 5 --warmup ${WARM:-1} --tol-run 0 --no-cpu-baseline --hbm-crops 0 > gpurun_out/geom_$g.json 2> gpurun_out/geom_$g.err || { echo "geom $g failed"; tail -20 gpurun_out/geom_$g.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/geom_$g.json'));print('geom $g', d['ms_per_step'], d['pdhg_iters_per_solve'], {k:v['ms'] for k,v in d['roofline']['kernels'].items()})"
done
