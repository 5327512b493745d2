#!/bin/bash
# Round 5: quick GPU check of the one-wave / loop paths after a small change
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "farmer_ph or persistent or host_loop or 10k or fused_pass or grouped_cached or seeded_iter0 or two_ranks or iteration_limit" > $O/pytest_r05_quick.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_r05_quick.log | tail -8
[ $rc -eq 0 ] || { grep -v "^frame" $O/pytest_r05_quick.log | tail -40; exit $rc; }
B="--no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0 --uc-scens 0"
for r in 1 2; do
  timeout -k 10 200 python -u bench.py $B > $O/f2_q$r.json 2> $O/f2_q$r.err || { echo "bench failed"; tail -20 $O/f2_q$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/f2_q$r.json'));print(d['ms_per_step'], d['ph_to_tol']['seconds'], d['ph_to_tol']['ph_iterations'], d['roofline']['kernels'])"
done
