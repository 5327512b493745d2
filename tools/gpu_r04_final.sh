#!/bin/bash
# Round-4 final check: the whole GPU suite, smoke(), the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/ > $O/pytest_gpu_final.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu_final.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_final.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke_final.log; exit 1; }
tail -3 $O/smoke_final.log
bash tools/archive/gpu_r04_bench.sh
