#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python tools/loop_prof.py 10000 50 200 > $O/loop_prof.txt 2>&1 || { echo "loop_prof failed"; tail -30 $O/loop_prof.txt; exit 1; }
cat $O/loop_prof.txt
