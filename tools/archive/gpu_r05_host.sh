#!/bin/bash
# Round 5: host_prof plain and under rocprofv3 --kernel-trace (same window)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/host_prof.py 10000 5 20 > $O/host_prof.txt 2>&1 || { tail -20 $O/host_prof.txt; exit 1; }
grep -v amdgpu.ids $O/host_prof.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace -d $O/ktr2 -o ktr --output-format csv -- python3 $R/tools/host_prof.py 10000 5 20 > $O/host_prof_rp.txt 2>&1 || { tail -20 $O/host_prof_rp.txt; exit 1; }
grep passes $O/host_prof_rp.txt
python3 $R/tools/trace_window.py $O/ktr2/ktr_kernel_trace.csv 5 20
