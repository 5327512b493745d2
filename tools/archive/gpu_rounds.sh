#!/bin/bash
# mid-size polish PDAS rounds at F3 iterations 30..34 (pinned rows)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for r in ${ROUNDS:-4 6}; do
  PHGPU_MID_POLISH_ROUNDS=$r timeout -k 10 250 python -u tools/mid_polish_prof.py 10000 100 30 4 > gpurun_out/rounds_$r.txt 2>&1 || { echo "rounds $r failed"; tail -5 gpurun_out/rounds_$r.txt; exit 1; }
  echo "== rounds $r"; grep -v -e Warn -e amdgpu.ids gpurun_out/rounds_$r.txt
done
