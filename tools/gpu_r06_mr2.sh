#!/bin/bash
# Round 6: 2 ranks (gloo) on one GPU, F2 only, cooperative launches forced
# on / off (PHGPU_COOP): two processes' cooperative launches on one device
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
for c in 0 1; do
  PHGPU_COOP=$c BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0 --uc-scens 0 \
    > $O/mr2_coop$c.json 2> $O/mr2_coop$c.err || { echo "mr coop $c failed"; tail -20 $O/mr2_coop$c.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/mr2_coop$c.json').read().strip().splitlines()[-1]);print('COOP=$c', d['n_gpus'], d['ms_per_step'], d['ph_to_tol']['seconds'], d['ph_to_tol']['ph_iterations'], d['ph_to_tol']['Eobj'])"
done
echo ALLDONE
