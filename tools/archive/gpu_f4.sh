#!/bin/bash
# F4 probe (farmer c=1000, 1000 scenarios: Iter0 + 3 PH iterations with the
# big_kernel's streaming rate), F3 polish with smaller regularisation, and
# the F2 bench with and without graph replay.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/f4_probe.py 1000 1000 3 > $O/f4_probe.txt 2>&1 || { echo "f4 probe failed"; tail -20 $O/f4_probe.txt; exit 1; }
cat $O/f4_probe.txt
for d in 1e-9 1e-10; do
  PHGPU_KKT_DELTA=$d timeout -k 10 200 python -u tools/mid_polish_prof.py 10000 100 30 4 > $O/midpol_d$d.txt 2>&1 || { echo "midpol $d failed"; tail -20 $O/midpol_d$d.txt; exit 1; }
  echo "delta $d"; cat $O/midpol_d$d.txt
done
for g in 1 0; do
  timeout -k 10 200 python -u bench.py --tol-run 0 --no-cpu-baseline --hbm-crops 0 --sslp-scens 0 --graphs $g > $O/bench_g$g.json 2> $O/bench_g$g.err || { echo "bench g$g failed"; tail -20 $O/bench_g$g.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_g$g.json')); print('graphs $g', d['ms_per_step'], d['roofline']['kernels'])"
done
