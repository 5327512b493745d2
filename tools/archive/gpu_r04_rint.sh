#!/bin/bash
# Row interleave: sslp / F3 phase clocks, then the whole GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
bash tools/gpu_r04_midprof.sh || exit 1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/ > $O/pytest_gpu_rint.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_gpu_rint.log | tail -70
exit $rc
