#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/tol_prof.py 10000 > $O/tol_prof.txt 2>&1 || { tail -20 $O/tol_prof.txt; exit 1; }
grep -v amdgpu.ids $O/tol_prof.txt
