#!/bin/bash
# Round 6: cooperative launches only with a spoke batch alive -- cylinder,
# team and multi-rank GPU tests, then the 2-rank default rehearsal (gloo,
# one GPU, every companion config)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "spin_the_wheel or async_spokes or uc_hub or big_teams or two_ranks or ragged or late_tail or fused_pass or collective" > $O/pytest_coop.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_coop.log | tail -16
[ $rc -eq 0 ] || exit 1
BENCH_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --no-cpu-baseline \
  > $O/mr2_default_b.json 2> $O/mr2_default_b.err || { echo "2-rank default bench failed"; grep -v amdgpu.ids $O/mr2_default_b.err | tail -30; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/mr2_default_b.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'ms', d['ms_per_step'], 'value', d['value'], 'tol', d['ph_to_tol']['seconds'], d['ph_to_tol']['ph_iterations'])
for k in ('hbm_config','f4_config','sslp_config'):
    print(k, d[k].get('ms_per_step'), d[k].get('ef_bracket',{}).get('ok'))
u=d['uc_config']; print('uc', u.get('ms_per_ph_iteration'), u.get('not_optimal_after'), u.get('lagrangian_bound'))
"
echo ALLDONE
