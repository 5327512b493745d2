#!/bin/bash
# F2 with the adaptive per-pass / persistent choice, then the default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
B="python bench.py --tol-run 1 --no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0 --uc-scens 0"
timeout -k 10 300 $B > $O/bench_f2_adapt.json 2> $O/bench_f2_adapt.err || { echo "bench failed"; tail -30 $O/bench_f2_adapt.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_f2_adapt.json')); print('adapt', d['ms_per_step'], d['ph_to_tol']['seconds'], d['ph_to_tol']['ph_iterations'], d['ph_to_tol']['Eobj'], d['roofline']['kernel'], d['roofline']['frac'])"
timeout -k 10 900 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; tail -30 $O/bench_default.err; exit 1; }
cat $O/bench_default.json | head -c 1500
