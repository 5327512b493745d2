#!/bin/bash
# One GPU call of experiments: mid-size polish PDAS rounds at F3 (10, 16
# against the default 6) and the big path's polish counters at F4 size
# (1,000 scenarios, c=1000, 2 PH iterations).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
ROUNDS="${ROUNDS:-6 10 16}" bash tools/gpu_rounds.sh || exit 1
timeout -k 10 300 python -u tools/big_polish_prof.py 1000 1000 2 > gpurun_out/bigpol_f4.txt 2>&1 || { echo "big failed"; tail -20 gpurun_out/bigpol_f4.txt; exit 1; }
cat gpurun_out/bigpol_f4.txt
