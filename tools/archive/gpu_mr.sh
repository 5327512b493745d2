#!/bin/bash
# bench.py --gpus 2 without a launcher, two ranks sharing the one GPU over gloo
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --scens 2000 --steps 10 --warmup 3 --no-cpu-baseline --hbm-crops 0 --tol-scens 2000 --cpu-scens 2000 > gpurun_out/mr.json 2> gpurun_out/mr.err || { echo "2-rank bench failed"; tail -20 gpurun_out/mr.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/mr.json'));print(d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'], d['ph_to_tol'])"
