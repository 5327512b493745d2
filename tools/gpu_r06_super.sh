#!/bin/bash
# Round 6: the device supernodal factor + solve on the UC pattern (one
# workgroup), per-level clocks (tests/native/super_gpu_check.hip).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
python tools/dump_pattern.py uc 1 0.2 0.3 0.5 > $O/pat_uc.txt || exit 1
timeout -k 10 120 tests/native/bin/super_gpu_check < $O/pat_uc.txt > $O/super_uc_r06.txt 2>&1 || exit 1
cat $O/super_uc_r06.txt
