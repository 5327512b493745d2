#!/bin/bash
# The big path's ILP sweeps: F4 Iter0 + PH iterations (f4_probe), UC at
# pdhg_tol 1e-6 (3 scenarios, 1 PH iteration).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/f4_probe.py 1000 1000 5 > $O/f4_probe_ilp.txt 2>&1 || { echo "f4 probe failed"; tail -30 $O/f4_probe_ilp.txt; exit 1; }
cat $O/f4_probe_ilp.txt
timeout -k 10 600 python -u tools/uc_probe.py 3 1 200000 1e-6 > $O/uc_probe3_tol6.txt 2>&1 || { echo "uc probe failed"; tail -30 $O/uc_probe3_tol6.txt; exit 1; }
grep -v '\.\.\.$' $O/uc_probe3_tol6.txt
