#!/bin/bash
# The big path's parity test + the mid-size tests its shared code touches,
# then the mid-size polish exit counters at F3 iterations 30-34.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "c1000 or c100 or infeasible or unbounded or sslp or graph_replay" > $O/pytest_big.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_big.log; exit 1; }
tail -3 $O/pytest_big.log
timeout -k 10 200 python -u tools/mid_polish_prof.py 10000 100 30 4 > $O/midpol_fix.txt 2>&1 || { echo "midpol failed"; tail -20 $O/midpol_fix.txt; exit 1; }
cat $O/midpol_fix.txt
