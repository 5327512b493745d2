#!/bin/bash
# F4 polish counters (16 scenarios), F2 graph replay vs eager twice, F3 with
# the 512-thread mid-size instances.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/big_polish_prof.py 16 1000 3 > $O/bigpol.txt 2>&1 || { echo "bigpol failed"; tail -20 $O/bigpol.txt; exit 1; }
cat $O/bigpol.txt
for r in 1 2; do for g in 1 0; do
  timeout -k 10 200 python -u bench.py --tol-run 0 --no-cpu-baseline --hbm-crops 0 --sslp-scens 0 --f4-scens 0 --graphs $g > $O/bench_g${g}_$r.json 2> $O/bench_g${g}_$r.err || { echo "bench g$g failed"; tail -20 $O/bench_g${g}_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_g${g}_$r.json')); print('graphs $g run $r', d['ms_per_step'])"
done; done
PHGPU_MID_GEOM=512 timeout -k 10 200 python -u tools/mid_polish_prof.py 10000 100 30 4 > $O/midpol_g512.txt 2>&1 || { echo "midpol 512 failed"; tail -20 $O/midpol_g512.txt; exit 1; }
cat $O/midpol_g512.txt
