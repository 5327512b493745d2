#!/bin/bash
# sslp_15_45_synthetic PH probe with and without pinned rows in the mid-size polish
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for v in 1 0; do
  PHGPU_MID_PIN=$v timeout -k 10 250 python -u tools/workload_probe.py sslp ${S:-10000} 0 10 > gpurun_out/sslp_pin$v.txt 2>&1 || { echo "pin $v failed"; tail -8 gpurun_out/sslp_pin$v.txt; exit 1; }
  echo "== pin $v"; grep -v -e Warn -e amdgpu.ids gpurun_out/sslp_pin$v.txt
done
