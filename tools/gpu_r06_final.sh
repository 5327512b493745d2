#!/bin/bash
# Round 6 end check (one GPU call): the whole GPU suite, smoke(), then the
# default bench line (TAG names the outputs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
T=${TAG:-r06_final}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/pytest_gpu_$T.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu_$T.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke_$T.log; exit 1; }
tail -1 $O/smoke_$T.log
timeout -k 10 900 python -u bench.py > $O/bench_$T.json 2> $O/bench_$T.err || { echo "bench failed"; tail -30 $O/bench_$T.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_$T.json'));print(d['ms_per_step'], d['ph_to_tol']['seconds'], d['hbm_config']['ms_per_step'], d['f4_config']['ms_per_step'], d['f4_config'].get('ef_bracket',{}).get('ok'), d['sslp_config']['ms_per_step']); print(json.dumps(d['uc_config']))"
exit $rc
