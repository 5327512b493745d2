#!/bin/bash
# Mid-size path phase launches one by one (sslp 10k, F3 10k): where the
# PH iteration's time goes and which scenarios hold each phase.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u tools/mid_phase_probe.py sslp 10000 5 4 > $O/midprobe_sslp.txt 2>&1 || { echo "sslp probe failed"; tail -30 $O/midprobe_sslp.txt; exit 1; }
cat $O/midprobe_sslp.txt
timeout -k 10 400 python -u tools/mid_phase_probe.py farmer100 10000 5 3 > $O/midprobe_f3.txt 2>&1 || { echo "f3 probe failed"; tail -30 $O/midprobe_f3.txt; exit 1; }
cat $O/midprobe_f3.txt
