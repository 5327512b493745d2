#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py"
timeout -k 10 600 $T -k "persistent_loop or host_loop_device_loop" > $O/pair_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/pair_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pair_tests.log
timeout -k 10 300 python tools/loop_prof.py 10000 50 200 > $O/loop_prof2.txt 2>&1 || { echo "loop_prof failed"; tail -30 $O/loop_prof2.txt; exit 1; }
cat $O/loop_prof2.txt
timeout -k 10 900 python bench.py > $O/bench_r04.json 2> $O/bench_r04.err || { echo "bench failed"; tail -30 $O/bench_r04.err; exit 1; }
cat $O/bench_r04.json
