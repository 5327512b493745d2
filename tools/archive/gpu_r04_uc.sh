#!/bin/bash
# UC LP relaxation probe on the GPU (3 scenarios, 2 PH iterations), then
# the F4 PH-to-tolerance run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/uc_probe.py 3 1 5000 > $O/uc_probe3.txt 2>&1 || { echo "uc probe failed"; tail -30 $O/uc_probe3.txt; exit 1; }
cat $O/uc_probe3.txt
