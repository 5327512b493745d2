#!/bin/bash
# two F2 headline runs back to back (noise check)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --tol-run 0 --no-cpu-baseline --hbm-crops 0 > gpurun_out/f2_$r.json 2> gpurun_out/f2_$r.err || { echo "run $r failed"; tail -10 gpurun_out/f2_$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/f2_$r.json'));print($r, d['ms_per_step'], d['value'], {k:v['ms'] for k,v in d['roofline']['kernels'].items()})"
done
