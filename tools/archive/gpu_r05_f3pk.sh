#!/bin/bash
# Round 5: F3 with the packed polish words compiled out past the VGPR budget
# (mid tests + the F3 line), then F4 PH to 1e-5
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "grouped_cached" > $O/pytest_r05_f3pk.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_r05_f3pk.log | tail -8
[ $rc -eq 0 ] || { grep -v "^frame" $O/pytest_r05_f3pk.log | tail -40; exit $rc; }
timeout -k 10 300 python -u bench.py --only f3 --no-cpu-baseline --tol-run 0 > $O/f3pk.json 2> $O/f3pk.err || { echo "f3 failed"; tail -20 $O/f3pk.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/f3pk.json'))['f3'];print('F3', d['ms_per_step'], d.get('iter0_seconds'), d['roofline'].get('kernel_ms'))"
timeout -k 10 300 python -u bench.py --only sslp --no-cpu-baseline --tol-run 0 > $O/sslppk.json 2> $O/sslppk.err || { echo "sslp failed"; tail -20 $O/sslppk.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/sslppk.json'))['sslp'];print('sslp', d['ms_per_step'])"
timeout -k 10 800 python -u tools/f4_to_tol.py 1000 1000 1e-5 30000 > $O/f4_to_tol_1e-5.json 2> $O/f4_to_tol_1e-5.log || { echo "f4 failed"; tail -5 $O/f4_to_tol_1e-5.log; exit 1; }
tail -2 $O/f4_to_tol_1e-5.log
cat $O/f4_to_tol_1e-5.json
