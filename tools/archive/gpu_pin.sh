#!/bin/bash
# Pinned-row slack test (PHGPU_MID_PIN=2) against plain pinning (1): F3
# polish counters at iterations 30-33 and the big polish at F4 size
# (1,000 scenarios, c=1000, 2 PH iterations).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for p in ${PINS:-1 2}; do
  PHGPU_MID_PIN=$p timeout -k 10 250 python -u tools/mid_polish_prof.py 10000 100 30 4 > gpurun_out/pin${p}_f3.txt 2>&1 || { echo "f3 pin $p failed"; tail -5 gpurun_out/pin${p}_f3.txt; exit 1; }
  echo "== F3 pin $p"; grep -v -e Warn -e amdgpu.ids gpurun_out/pin${p}_f3.txt
done
for p in ${PINS:-1 2}; do
  PHGPU_MID_PIN=$p timeout -k 10 300 python -u tools/big_polish_prof.py 1000 1000 3 > gpurun_out/pin${p}_f4.txt 2>&1 || { echo "f4 pin $p failed"; tail -5 gpurun_out/pin${p}_f4.txt; exit 1; }
  echo "== F4 pin $p"; grep -v -e Warn -e amdgpu.ids gpurun_out/pin${p}_f4.txt
done
