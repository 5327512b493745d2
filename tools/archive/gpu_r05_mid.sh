#!/bin/bash
# Round 5: mid-size phase launches by PDAS round limit (sslp 10k, F3 10k)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for r in 6 10 16; do
  for w in sslp farmer100; do
    PHGPU_MID_POLISH_ROUNDS=$r timeout -k 10 300 python -u tools/mid_phase_probe.py $w 10000 5 3 > $O/mid_phases_${w}_r$r.txt 2>&1 || { tail -20 $O/mid_phases_${w}_r$r.txt; exit 1; }
    echo "== $w rounds $r"; grep -v amdgpu.ids $O/mid_phases_${w}_r$r.txt | tail -3 | cut -c1-200
  done
done
