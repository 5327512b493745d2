#!/bin/bash
# Round 6: F4 big polish at HEAD -- exit counters per PH iteration, the phase
# launches one by one, then the F4 and F2 PMC profiles (tools/gpu_r06_prof.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/big_polish_prof.py 1000 1000 8 > $O/f4_polish_counters_aset.txt 2>&1 || { echo "big_polish_prof failed"; tail -20 $O/f4_polish_counters_aset.txt; exit 1; }
grep -v amdgpu.ids $O/f4_polish_counters_aset.txt | cut -c1-400
timeout -k 10 300 python3 -u tools/mid_phase_probe.py farmer1000 1000 5 3 > $O/f4_phases.txt 2>&1 || { echo "phase probe failed"; tail -20 $O/f4_phases.txt; exit 1; }
grep -v amdgpu.ids $O/f4_phases.txt | cut -c1-600
bash tools/gpu_r06_prof.sh r06 "f4 f2" || exit 1
