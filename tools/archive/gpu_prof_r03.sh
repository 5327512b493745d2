#!/bin/bash
# Round-3 measurement call: per-workload rocprofv3 profiles (tools/gpu_full.sh),
# the mid-size polish exit counters at F3 iterations 30-34 (4 and 6 PDAS
# rounds), the host issue time of one device-loop pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/mid_polish_prof.py 10000 100 30 4 > $O/midpol_r4.txt 2>&1 || { echo "midpol 4 failed"; tail -20 $O/midpol_r4.txt; exit 1; }
cat $O/midpol_r4.txt
PHGPU_MID_POLISH_ROUNDS=6 timeout -k 10 200 python -u tools/mid_polish_prof.py 10000 100 30 4 > $O/midpol_r6.txt 2>&1 || { echo "midpol 6 failed"; tail -20 $O/midpol_r6.txt; exit 1; }
cat $O/midpol_r6.txt
timeout -k 10 200 python -u tools/host_issue.py 10000 400 > $O/host_issue.txt 2>&1 || { echo "host issue failed"; tail -20 $O/host_issue.txt; exit 1; }
cat $O/host_issue.txt
bash tools/gpu_full.sh r03
