#!/bin/bash
# Round 5: the whole GPU suite, then the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/pytest_gpu_r05.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu_r05.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench_r05.json 2> $O/bench_r05.err || { echo "bench failed"; tail -30 $O/bench_r05.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_r05.json'));print(d['ms_per_step'], d['ph_to_tol']['seconds'], d['vs_cpu'], d['hbm_config']['ms_per_step'], d['f4_config']['ms_per_step'], d['f4_config'].get('iter0_seconds'), d['sslp_config']['ms_per_step'], d['uc_config'] and d['uc_config'].get('ms_per_ph_iter'))"
