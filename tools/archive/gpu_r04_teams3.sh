#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py"
timeout -k 10 900 $T -k "big_teams or hard_iter0 or c1000_big_path or uc_lp_relaxation" > $O/teams_tests3.log 2>&1 || { echo "tests failed"; tail -60 $O/teams_tests3.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/teams_tests3.log
timeout -k 10 300 python -u tools/f4_probe.py 1000 1000 5 > $O/f4_probe_teams3.txt 2>&1 || { echo "f4 probe failed"; tail -30 $O/f4_probe_teams3.txt; exit 1; }
cat $O/f4_probe_teams3.txt
timeout -k 10 600 python -u tools/uc_probe.py 3 1 1000000 > $O/uc_probe3_teams3.txt 2>&1 || { echo "uc probe failed"; tail -30 $O/uc_probe3_teams3.txt; exit 1; }
grep -v '\.\.\.$' $O/uc_probe3_teams3.txt
