#!/bin/bash
# Round 5: the supernodal LDL' (kkt_super.h / solve_super.inc): F4-shape
# parity with it forced on, then the UC probe (3 scenarios, 2 PH iterations).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
PHGPU_KKT_SUPER=1 timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "c1000" > $O/pytest_r05_super_f4.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_r05_super_f4.log | tail -10
[ $rc -eq 0 ] || { grep -v "^frame" $O/pytest_r05_super_f4.log | tail -50; exit $rc; }
PHGPU_VERBOSE=1 timeout -k 10 400 python -u tools/uc_probe.py 3 2 200000 1e-9 > $O/uc_super_probe.log 2>&1; rc=$?
tail -30 $O/uc_super_probe.log
exit $rc
