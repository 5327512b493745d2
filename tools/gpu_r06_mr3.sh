#!/bin/bash
# Round 6 (end): the default line on 2 gloo ranks on the box's one GPU, the
# UC cylinders left out (two processes' plain team launches on one device
# can hold each other's teams; one rank per GPU in the driver's runs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
BENCH_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --no-cpu-baseline --uc-scens 0 \
  > $O/mr2_default_c.json 2> $O/mr2_default_c.err || { echo "2-rank bench failed"; grep -v amdgpu.ids $O/mr2_default_c.err | tail -30; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/mr2_default_c.json').read().strip().splitlines()[-1])
print('n_gpus', d['n_gpus'], 'ms', d['ms_per_step'], 'value', d['value'], 'tol', d['ph_to_tol']['seconds'], d['ph_to_tol']['ph_iterations'])
for k in ('hbm_config','f4_config','sslp_config'):
    print(k, d[k].get('ms_per_step'))
"
echo ALLDONE
