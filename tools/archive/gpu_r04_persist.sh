#!/bin/bash
# Round 4: the persistent device loop (loop_kernel) on the GPU: its parity
# tests against the per-pass kernels and the 10k golden trajectory, then the
# F2 headline with and without it (PHGPU_PERSIST=0), then its rocprof stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py"
timeout -k 10 600 $T -k "persistent_loop or variable_probability" > $O/persist_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/persist_tests.log; exit 1; }
tail -8 $O/persist_tests.log
B="python bench.py --steps 200 --warmup 20 --tol-run 0 --no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0"
timeout -k 10 300 $B > $O/bench_persist.json 2> $O/bench_persist.err || { echo "bench failed"; tail -30 $O/bench_persist.err; exit 1; }
cat $O/bench_persist.json
PHGPU_PERSIST=0 timeout -k 10 300 $B > $O/bench_perpass.json 2> $O/bench_perpass.err || { echo "bench perpass failed"; tail -30 $O/bench_perpass.err; exit 1; }
cat $O/bench_perpass.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/persist_stats -o run -- python3 bench.py --steps 200 --warmup 20 --tol-run 0 --no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0 > $O/persist_stats.json 2> $O/persist_stats.log || { echo "rocprof failed"; tail -30 $O/persist_stats.log; exit 1; }
head -12 $(find $O/persist_stats -name '*kernel_stats.csv' | head -1)
