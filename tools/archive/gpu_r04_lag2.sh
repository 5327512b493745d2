#!/bin/bash
# Lagged persistent loop, second form: parity tests and the loop profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py"
timeout -k 10 600 $T -k "persistent_loop or farmer_10k_ph_trajectory" > $O/lag_tests.log 2>&1 || { echo "tests failed"; grep -E "assert|Error|FAILED" $O/lag_tests.log | head -20; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/lag_tests.log
timeout -k 10 300 python tools/loop_prof.py 10000 50 200 > $O/loop_prof_lag.txt 2>&1 || { echo "loop_prof failed"; tail -30 $O/loop_prof_lag.txt; exit 1; }
grep -v amdgpu.ids $O/loop_prof_lag.txt
B="python bench.py --tol-run 1 --no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0 --uc-scens 0"
timeout -k 10 300 $B > $O/bench_f2_lag_adapt.json 2> $O/bench_f2_lag_adapt.err || { echo "bench failed"; tail -30 $O/bench_f2_lag_adapt.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_f2_lag_adapt.json')); print('adapt', d['ms_per_step'], d['ph_to_tol']['seconds'], d['ph_to_tol']['ph_iterations'], d['ph_to_tol']['Eobj'])"
