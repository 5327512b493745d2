#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py"
timeout -k 10 900 $T -k "big_teams or hard_iter0 or c1000_big_path or uc_lp_relaxation or infeasible_scenario or unbounded" > $O/teams_tests4.log 2>&1 || { echo "tests failed"; tail -60 $O/teams_tests4.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/teams_tests4.log
for r in 1 2; do
timeout -k 10 300 python -u tools/uc_probe.py 3 0 1000000 > $O/uc_det$r.txt 2>&1 || { echo "uc probe failed"; tail -30 $O/uc_det$r.txt; exit 1; }
grep "Iter0" $O/uc_det$r.txt
done
timeout -k 10 300 python -u tools/f4_probe.py 1000 1000 5 > $O/f4_probe_teams5.txt 2>&1 || { echo "f4 probe failed"; tail -30 $O/f4_probe_teams5.txt; exit 1; }
cat $O/f4_probe_teams5.txt
