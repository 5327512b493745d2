#!/bin/bash
# Round 5: seeded Iter0 by the number of representatives (F2 10k)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for r in 8 32 128 512; do
  PHGPU_PRIME_REPS=$r timeout -k 10 200 python -u tools/tol_prof.py 10000 > $O/tol_prof_reps$r.txt 2>&1 || { tail -20 $O/tol_prof_reps$r.txt; exit 1; }
  echo "== reps $r"; grep -E "Iter0 solve|^rep 1" $O/tol_prof_reps$r.txt | tail -2
done
