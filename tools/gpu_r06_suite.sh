#!/bin/bash
# Round 6: the whole GPU suite, the supernodal factor's clocks on UC, then
# the default bench line (TAG names the outputs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
T=${TAG:-r06}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/pytest_gpu_$T.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu_$T.log | tail -20
[ $rc -eq 0 ] || exit $rc
if [ -z "$NOSUPER" ]; then
  python tools/dump_pattern.py uc 1 0.2 0.3 0.5 > $O/pat_uc.txt || exit 1
  timeout -k 10 120 tests/native/bin/super_gpu_check < $O/pat_uc.txt > $O/super_uc_$T.txt 2>&1 || exit 1
  tail -2 $O/super_uc_$T.txt | cut -c1-400
fi
timeout -k 10 600 python -u bench.py > $O/bench_$T.json 2> $O/bench_$T.err || { echo "bench failed"; tail -30 $O/bench_$T.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_$T.json'));print(d['ms_per_step'], d['ph_to_tol']['seconds'], d['hbm_config']['ms_per_step'], d['f4_config']['ms_per_step'], d['f4_config'].get('ef_bracket'), d['sslp_config']['ms_per_step'], d['uc_config'] and d['uc_config'].get('ms_per_ph_iteration'))"
