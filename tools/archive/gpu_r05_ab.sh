#!/bin/bash
# Round 5: cooperative vs plain launches (F2 PH to 1e-4), the CPU-baseline
# rank sweep, F4 PH to 1e-5.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
B="--no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0 --uc-scens 0"
for c in 1 0 1 0; do
  PHGPU_COOP=$c timeout -k 10 200 python -u bench.py $B > $O/ab_coop$c.json 2> $O/ab_coop$c.err || { echo "bench coop=$c failed"; tail -20 $O/ab_coop$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_coop$c.json'));print('coop', $c, d['ms_per_step'], d['ph_to_tol']['seconds'], d['ph_to_tol']['ph_iterations'])"
done
timeout -k 10 500 python -u tools/cpu_ranks_sweep.py 30 16 32 64 128 > $O/cpu_ranks_sweep.json 2> $O/cpu_ranks_sweep.err || { echo "sweep failed"; tail -5 $O/cpu_ranks_sweep.err; }
tail -4 $O/cpu_ranks_sweep.err
if [ "${F4TOL:-1}" = "1" ]; then
timeout -k 10 600 python -u tools/f4_to_tol.py 1000 1000 1e-5 60000 > $O/f4_to_tol_1e-5.json 2> $O/f4_to_tol_1e-5.log || { echo "f4 failed"; tail -5 $O/f4_to_tol_1e-5.log; exit 1; }
cat $O/f4_to_tol_1e-5.json
fi
