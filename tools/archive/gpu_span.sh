#!/bin/bash
# F3 companion (warmup 5, 5 steps) with the default primal-weight span and with a QP-only span
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for sp in 4 8 16; do
  PHGPU_MID_POLISH_ROUNDS=$sp timeout -k 10 300 python -u bench.py --crops 100 --steps 5 --warmup 5 --tol-run 0 --no-cpu-baseline --hbm-crops 0 > gpurun_out/span_$sp.json 2> gpurun_out/span_$sp.err || { echo "span $sp failed"; tail -10 gpurun_out/span_$sp.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/span_$sp.json'));print('span $sp', d['ms_per_step'], d['pdhg_iters_per_solve'])"
  grep -c "Solve failed" gpurun_out/span_$sp.err || true
done
