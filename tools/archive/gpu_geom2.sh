#!/bin/bash
# F2 ms per PH iteration under launch-geometry hooks
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for v in "41 64" "81 64" "41 8" "81 8"; do
  set -- $v
  PHGPU_AS_GEOM=$1 PHGPU_TAIL_GRID=$2 timeout -k 10 200 python -u bench.py --tol-run 0 --no-cpu-baseline --hbm-crops 0 > gpurun_out/g2.json 2> gpurun_out/g2.err || { echo "run $v failed"; tail -10 gpurun_out/g2.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/g2.json'));print('as $1 tail $2', d['ms_per_step'], {k:v['ms'] for k,v in d['roofline']['kernels'].items()})"
done
