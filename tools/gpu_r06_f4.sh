#!/bin/bash
# Round 6: the big path with the scenario-slowest copies (x, y, PH terms):
# its GPU tests, the UC cylinders test, F4's PMC profile at HEAD, then the
# default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ -k "c1000 or uc_hub or teams or collective or bundled" > $O/pytest_gpu_r06_big.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_gpu_r06_big.log | tail -30
# (test failures: rc 1; anything else -- a crash, a timeout -- ends the call here)
[ $rc -le 1 ] || exit $rc
bash tools/gpu_r06_prof.sh r06 "f4" || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_r06b.json 2> $O/bench_r06b.err || { echo "bench failed"; tail -30 $O/bench_r06b.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_r06b.json'));print(d['ms_per_step'], d['ph_to_tol']['seconds'], d['hbm_config']['ms_per_step'], d['f4_config']['ms_per_step'], d['f4_config']['iter0_s'], d['f4_config'].get('ef_bracket'), d['sslp_config']['ms_per_step']); print(json.dumps(d['uc_config']))"
exit $rc
