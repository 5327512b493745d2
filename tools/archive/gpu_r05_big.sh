#!/bin/bash
# Round 5: the 512-thread big polish: big-path parity tests, F4 companion;
# F3 with / without the packed pattern words (pk16).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "c1000 or uc_lp or teams or async_spokes or supernodal" > $O/pytest_r05_big.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_r05_big.log | tail -20
[ $rc -eq 0 ] || { grep -v "^frame" $O/pytest_r05_big.log | tail -40; exit $rc; }
timeout -k 10 200 python -u bench.py --only f4 > $O/only_f4.json 2> $O/only_f4.err || { echo "f4 failed"; tail -20 $O/only_f4.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/only_f4.json'))['f4'];print('F4', d['ms_per_step'], d['iter0_s'], d['roofline']['kernel_ms'], d['roofline']['polish_ms'], d['roofline']['launches'], d['roofline']['polish_launches'])"
for pk in 1 0; do
  PHGPU_MID_PK16=$pk timeout -k 10 200 python -u bench.py --only f3 > $O/only_f3_pk$pk.json 2> $O/only_f3_pk$pk.err || { echo "f3 failed"; tail -20 $O/only_f3_pk$pk.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/only_f3_pk$pk.json'))['f3'];print('F3 pk16=$pk', d['ms_per_step'], d['iter0_s'], d['roofline']['kernel_ms'])"
done
