#!/bin/bash
# Round 5: F4 PH to conv < 1e-5 (limit 30,000 iterations): how the bracket
# [post_solve_bound, x-bar objective] around the published EF narrows
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 1000 python -u tools/f4_to_tol.py 1000 1000 1e-5 30000 > $O/f4_to_tol_1e-5.json 2> $O/f4_to_tol_1e-5.log || { echo "f4 failed"; tail -5 $O/f4_to_tol_1e-5.log; exit 1; }
tail -3 $O/f4_to_tol_1e-5.log
cat $O/f4_to_tol_1e-5.json
