#!/bin/bash
# Round 5 end: the whole GPU suite, smoke(), the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/pytest_gpu_final.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu_final.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_final.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke_final.log; exit 1; }
tail -1 $O/smoke_final.log
timeout -k 10 400 python -u bench.py > $O/bench_r05_final.json 2> $O/bench_r05_final.err || { echo "bench failed"; tail -30 $O/bench_r05_final.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_r05_final.json'));print(d['value'], d['ms_per_step'], d['ph_to_tol']['seconds'], d['ph_to_tol']['ph_iterations'], d['vs_cpu']['ph_to_tol_speedup'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic'], d['hbm_config']['ms_per_step'], d['f4_config']['ms_per_step'], d['sslp_config']['ms_per_step'])"
if [ "${F4AB:-0}" = "1" ]; then
  PHGPU_MID_POLISH_ROUNDS=10 timeout -k 10 400 python -u bench.py --only f4 --no-cpu-baseline --tol-run 0 > $O/f4r_10.json 2> $O/f4r_10.err || { echo "f4 failed"; tail -20 $O/f4r_10.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/f4r_10.json'))['f4'];print('F4 rounds 10', d['ms_per_step'])"
fi
