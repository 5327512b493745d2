#!/bin/bash
# Mid-size geometry and polish / PDHG phase clocks at F3 and sslp.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python tools/mid_polish_prof.py 10000 100 6 5 > $O/midprof_f3.txt 2>&1 || { echo "f3 failed"; tail -30 $O/midprof_f3.txt; exit 1; }
grep -v amdgpu.ids $O/midprof_f3.txt
timeout -k 10 400 python tools/mid_polish_prof.py 10000 0 6 5 > $O/midprof_sslp.txt 2>&1 || { echo "sslp failed"; tail -30 $O/midprof_sslp.txt; exit 1; }
grep -v amdgpu.ids $O/midprof_sslp.txt
