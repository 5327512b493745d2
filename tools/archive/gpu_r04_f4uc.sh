#!/bin/bash
# F4 PH to tolerance against the published EF, then the UC LP relaxation
# (3 scenarios) with the full PDHG budget.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 950 python -u tools/f4_to_tol.py 1000 1000 1e-4 15000 > $O/f4tol.json 2> $O/f4tol.err || { echo "F4 to tol failed"; tail -30 $O/f4tol.err; exit 1; }
tail -5 $O/f4tol.err
cat $O/f4tol.json
timeout -k 10 700 python -u tools/uc_probe.py 3 1 200000 > $O/uc_probe3_full.txt 2>&1 || { echo "uc probe failed"; tail -30 $O/uc_probe3_full.txt; exit 1; }
cat $O/uc_probe3_full.txt
