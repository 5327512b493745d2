#!/bin/bash
# Round 5: loop_kernel phase clocks (LP_ARGS: S START NIT, default the bench
# window) and the per-pass polish_kernel's phase clocks in the same window
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/loop_prof.py ${LP_ARGS:-10000 5 20} > $O/loop_prof_lp.txt 2>&1 || { tail -20 $O/loop_prof_lp.txt; exit 1; }
grep -v amdgpu.ids $O/loop_prof_lp.txt
PHGPU_PERSIST=0 timeout -k 10 200 python -u tools/polish_prof.py 10000 1 5 20 > $O/polprof_lp.txt 2>&1 || { tail -20 $O/polprof_lp.txt; exit 1; }
grep -v amdgpu.ids $O/polprof_lp.txt
