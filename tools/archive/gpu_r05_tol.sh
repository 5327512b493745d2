#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for ch in 16 64 256; do
  timeout -k 10 200 python -u tools/tol_prof.py 10000 $ch > $O/tol_prof_c$ch.txt 2>&1 || { tail -20 $O/tol_prof_c$ch.txt; exit 1; }
  echo "== chunk $ch"; grep -v amdgpu.ids $O/tol_prof_c$ch.txt | tail -7
done
