#!/bin/bash
# Round 5: the device supernodal factor + solve (one workgroup) against the
# sparse KKT on the UC / F4 / sslp patterns (tests/native/super_gpu_check.hip).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
for spec in ${SPECS:-"sslp 1 0.2 0.3 0.5" "farmer100 2 0.3 0.3 0.5" "farmer1000 1 0.2 0.3 0.5" "uc 1 0.2 0.3 0.5"}; do
  set -- $spec
  python tools/dump_pattern.py $spec > $O/pat_$1.txt || exit 1
  echo "== $spec"
  timeout -k 10 120 tests/native/bin/super_gpu_check < $O/pat_$1.txt || exit 1
done
