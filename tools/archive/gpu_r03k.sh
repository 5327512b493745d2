#!/bin/bash
# Full GPU parity suite at the 512-thread default, big-polish counters with
# a capped grid (work-queue reuse), F3 / sslp timing at the new default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_k.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_gpu_k.log; exit 1; }
tail -3 $O/pytest_gpu_k.log
PHGPU_MID_GRID=4 timeout -k 10 300 python -u tools/big_polish_prof.py 16 1000 3 > $O/bigpol_g4.txt 2>&1 || { echo "bigpol failed"; tail -20 $O/bigpol_g4.txt; exit 1; }
cat $O/bigpol_g4.txt
timeout -k 10 200 python -u tools/mid_polish_prof.py 10000 100 30 4 > $O/midpol_512def.txt 2>&1 || { echo "midpol failed"; tail -20 $O/midpol_512def.txt; exit 1; }
cat $O/midpol_512def.txt
timeout -k 10 300 python -u bench.py --tol-run 0 --no-cpu-baseline --f4-scens 0 > $O/bench_k.json 2> $O/bench_k.err || { echo "bench failed"; tail -20 $O/bench_k.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_k.json')); print('F2', d['ms_per_step'], 'F3', d['hbm_config']['ms_per_step'], d['hbm_config']['roofline']['kernel_ms'], 'sslp', d['sslp_config']['ms_per_step'])"
