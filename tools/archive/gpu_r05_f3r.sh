#!/bin/bash
# Round 5: mid-size polish rounds by K/n: mid tests, F3 / sslp lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "c100 or mid or sslp or c1000" > $O/pytest_r05_f3r.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_r05_f3r.log | tail -8
[ $rc -eq 0 ] || { grep -v "^frame" $O/pytest_r05_f3r.log | tail -40; exit $rc; }
timeout -k 10 300 python -u bench.py --only f3 --no-cpu-baseline --tol-run 0 > $O/f3r.json 2> $O/f3r.err || { echo "f3 failed"; tail -20 $O/f3r.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/f3r.json'))['f3'];print('F3', d['ms_per_step'], d['roofline'].get('kernel_ms'))"
timeout -k 10 300 python -u bench.py --only sslp --no-cpu-baseline --tol-run 0 > $O/sslpr.json 2> $O/sslpr.err || { echo "sslp failed"; tail -20 $O/sslpr.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/sslpr.json'))['sslp'];print('sslp', d['ms_per_step'])"
