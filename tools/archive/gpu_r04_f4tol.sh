#!/bin/bash
# F4 PH to convergence against the published EF (tools/f4_to_tol.py); a
# small farmer run first checks the script end to end.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 150 python -u tools/f4_to_tol.py 30 1 1e-4 5000 > $O/f4tol_small.json 2> $O/f4tol_small.err || { echo "small run failed"; tail -20 $O/f4tol_small.err; exit 1; }
cat $O/f4tol_small.json
timeout -k 10 950 python -u tools/f4_to_tol.py 1000 1000 1e-4 15000 > $O/f4tol.json 2> $O/f4tol.err || { echo "F4 to tol failed"; tail -30 $O/f4tol.err; exit 1; }
tail -5 $O/f4tol.err
cat $O/f4tol.json
