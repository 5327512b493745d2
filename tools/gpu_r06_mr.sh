#!/bin/bash
# Round 6: the DEFAULT bench line (every companion config: F3, F4 with its
# EF bracket, sslp, UC cylinders) on 2 ranks -- gloo, both on the box's one
# GPU -- as the driver's scaling run will start it (torch.distributed.run)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
BENCH_DIST_BACKEND=gloo timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --no-cpu-baseline \
  > $O/mr2_default.json 2> $O/mr2_default.err || { echo "2-rank default bench failed"; grep -v amdgpu.ids $O/mr2_default.err | tail -30; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/mr2_default.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'ms', d['ms_per_step'], 'value', d['value'], 'tol', d['ph_to_tol']['seconds'], d['ph_to_tol']['ph_iterations'])
for k in ('hbm_config','f4_config','sslp_config'):
    print(k, d[k].get('ms_per_step'), d[k].get('workload','')[:80], d[k].get('ef_bracket',{}).get('ok'))
u=d['uc_config']; print('uc', u.get('ms_per_ph_iteration'), u.get('not_optimal_after'), u.get('lagrangian_bound'), u.get('workload','')[:70])
"
echo ALLDONE
