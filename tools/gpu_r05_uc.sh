#!/bin/bash
# Round 5: UC LP relaxation at 64 scenarios on one GPU (PDHG-only big path on
# teams): Iter0 and one PH iteration (tools/uc_probe.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 1100 python -u tools/uc_probe.py 64 1 > $O/uc_probe_64.txt 2>&1 || { tail -20 $O/uc_probe_64.txt; exit 1; }
grep -v "\.\.\.$" $O/uc_probe_64.txt | tail -12
