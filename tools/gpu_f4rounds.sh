#!/bin/bash
# F4 (farmer c=1000, 1,000 scenarios) bench line at several PDAS round limits
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for r in ${ROUNDS:-6 10 16}; do
  PHGPU_MID_POLISH_ROUNDS=$r timeout -k 10 300 python -u bench.py --hbm-crops 0 --sslp-scens 0 --no-cpu-baseline --tol-run 0 --scens 1000 --steps 5 --warmup 5 --f4-scens 1000 > gpurun_out/bench_f4_r$r.json 2> gpurun_out/bench_f4_r$r.err || { echo "rounds $r failed"; tail -5 gpurun_out/bench_f4_r$r.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_f4_r$r.json').read().strip().splitlines()[-1])['f4_config']; r=d['roofline']; print('rounds $r', d['ms_per_step'], 'ms/step; pdhg steps/solve', d['pdhg_steps_per_solve'], 'max', d['pdhg_steps_max'], 'big_kernel', r['kernel_ms'], 'ms /', r['launches'], 'polish', r['polish_ms'], 'ms /', r['polish_launches'])"
done
