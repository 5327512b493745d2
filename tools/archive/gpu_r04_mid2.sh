#!/bin/bash
# Mid-size probes, then the mid-size / polish GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
bash tools/gpu_r04_midprof.sh || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/ -k "sslp or c100 or mid_path or hydro or infeasible or unbounded or iteration_limit or large_valued or c1000 or uc_lp" > $O/pytest_gpu_mid2.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_gpu_mid2.log | tail -40
exit $rc
