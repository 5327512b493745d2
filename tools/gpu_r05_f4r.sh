#!/bin/bash
# Round 5: F4 polish rounds (the warm prox-QP polish) vs PH-iteration time.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
for r in 6 12 20; do
  echo "== rounds $r"
  PHGPU_MID_POLISH_ROUNDS=$r timeout -k 10 200 python -u tools/big_polish_prof.py 1000 1000 5 > $O/f4_rounds$r.txt 2>&1 || { tail -20 $O/f4_rounds$r.txt; exit 1; }
  grep "PH iteration" $O/f4_rounds$r.txt | cut -c1-400
done
