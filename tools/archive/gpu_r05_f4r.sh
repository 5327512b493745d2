#!/bin/bash
# Round 5: F4 line at the big polish's default rounds and at 10
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
for r in def 10; do
  if [ $r = def ]; then unset PHGPU_MID_POLISH_ROUNDS; else export PHGPU_MID_POLISH_ROUNDS=$r; fi
  timeout -k 10 400 python -u bench.py --only f4 --no-cpu-baseline --tol-run 0 > $O/f4r_$r.json 2> $O/f4r_$r.err || { echo "f4 failed"; tail -20 $O/f4r_$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/f4r_$r.json'))['f4'];print('F4 rounds $r', d['ms_per_step'], d.get('iter0_seconds'), d['roofline'].get('kernel_ms'))"
done
