#!/bin/bash
# Round 5: last check of the final binary: the one-wave / loop tests and smoke()
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "farmer_ph or persistent or host_loop or 10k or fused_pass or grouped_cached or seeded_iter0 or two_ranks or iteration_limit or c100 or sslp" > $O/pytest_r05_last.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_r05_last.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_last.log 2>&1 || { tail -20 $O/smoke_last.log; exit 1; }
tail -1 $O/smoke_last.log
