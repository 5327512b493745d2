#!/bin/bash
# Round 5: F2 kernel timeline (rocprofv3 --kernel-trace) of the bench's timed
# window (passes 6..25, no events): per-kernel durations and the gaps
# between consecutive dispatches (tools/trace_window.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace -d $O/ktr -o ktr --output-format csv -- python3 $R/bench.py --no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0 --uc-scens 0 --tol-run 0 > $O/ktr.log 2>&1 || { tail -20 $O/ktr.log; exit 1; }
python3 $R/tools/trace_window.py $O/ktr/ktr_kernel_trace.csv
