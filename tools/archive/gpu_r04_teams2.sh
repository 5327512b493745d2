#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py"
timeout -k 10 600 $T -k "big_teams" > $O/teams_tests2.log 2>&1 || { echo "tests failed"; tail -60 $O/teams_tests2.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/teams_tests2.log
timeout -k 10 300 python -u tools/f4_probe.py 1000 1000 5 > $O/f4_probe_teams.txt 2>&1 || { echo "f4 probe failed"; tail -30 $O/f4_probe_teams.txt; exit 1; }
cat $O/f4_probe_teams.txt
timeout -k 10 600 python -u tools/uc_probe.py 3 2 2000000 > $O/uc_probe3_teams.txt 2>&1 || { echo "uc probe failed"; tail -30 $O/uc_probe3_teams.txt; exit 1; }
grep -v '\.\.\.$' $O/uc_probe3_teams.txt
