#!/bin/bash
# Round 6: the big path's long-line threshold (PHGPU_BIG_LONG 32 / 16 / 8):
# UC probe (2 scenarios, no spoke: Iter0 + 2 PH iterations) and F4
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
for L in 32 16 8; do
  PHGPU_BIG_LONG=$L timeout -k 10 300 python3 -u tools/uc_probe.py 2 2 400000 > $O/uc_probe_long$L.txt 2>&1 || { echo "uc probe $L failed"; tail -5 $O/uc_probe_long$L.txt; exit 1; }
  echo "== BIG_LONG=$L"; grep -E "Iter0 [0-9.]+ s|PH iteration" $O/uc_probe_long$L.txt | cut -c1-160
  PHGPU_BIG_LONG=$L timeout -k 10 300 python3 bench.py --tol-run 0 --no-cpu-baseline --only f4 --hbm-steps 5 --f4-bracket 0 > $O/f4_long$L.json 2> $O/f4_long$L.log || { echo "f4 $L failed"; tail -20 $O/f4_long$L.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/f4_long$L.json'))['f4'];print('F4 long $L', d['ms_per_step'], d['iter0_s'], d['roofline'].get('polish_ms'), d['roofline'].get('kernel_ms'))"
done
echo ALLDONE
