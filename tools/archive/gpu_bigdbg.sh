#!/bin/bash
# The big path on F3's shape (PHGPU_FORCE_BIG=1) against the mid-size path:
# polish exit counters over Iter0 and 3 PH iterations, 16 scenarios.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/big_polish_prof.py 16 100 3 > $O/pol_mid_c100.txt 2>&1 || { echo "mid failed"; tail -20 $O/pol_mid_c100.txt; exit 1; }
echo mid; cat $O/pol_mid_c100.txt
PHGPU_FORCE_BIG=1 timeout -k 10 200 python -u tools/big_polish_prof.py 16 100 3 > $O/pol_big_c100.txt 2>&1 || { echo "big failed"; tail -20 $O/pol_big_c100.txt; exit 1; }
echo big; cat $O/pol_big_c100.txt
