#!/bin/bash
# Round 5: the multi-rank per-pass path with the fused solve: the two-rank
# GPU tests, a 2-rank gloo bench rehearsal on one GPU (fused / not)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "two_ranks or ragged or farmer_ph or persistent" > $O/pytest_r05_mr.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_r05_mr.log | tail -8
[ $rc -eq 0 ] || { grep -v "^frame" $O/pytest_r05_mr.log | tail -40; exit $rc; }
for mode in 1 0; do
  PHGPU_FUSED=$mode BENCH_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0 --uc-scens 0 \
    > $O/mr_$mode.json 2> $O/mr_$mode.err || { echo "mr bench failed"; tail -20 $O/mr_$mode.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/mr_$mode.json').read().strip().splitlines()[-1]);print('fused=$mode', d['n_gpus'], d['ms_per_step'], d['ph_to_tol']['seconds'], d['ph_to_tol']['ph_iterations'], d['ph_to_tol']['Eobj'])"
done
