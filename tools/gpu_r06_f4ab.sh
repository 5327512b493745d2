#!/bin/bash
# Round 6: F4 A/B of the big polish (the call-free instance; warm prox-QP
# classification by thresholds vs the PDAS rule): polish exit counters
# (tools/big_polish_prof.py) and the bench's F4 line, then the UC cylinders
# test and the big-path GPU tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
for pd in 0 1; do
  PHGPU_BIG_QP_PDAS=$pd timeout -k 10 300 python3 tools/big_polish_prof.py 1000 1000 4 > $O/f4_polprof_pdas$pd.txt 2>&1 || { echo "polprof $pd failed"; tail -20 $O/f4_polprof_pdas$pd.txt; exit 1; }
  grep -E "PH iteration" $O/f4_polprof_pdas$pd.txt | cut -c1-400
  PHGPU_BIG_QP_PDAS=$pd timeout -k 10 300 python3 bench.py --tol-run 0 --no-cpu-baseline --only f4 --hbm-steps 5 --f4-bracket 0 > $O/f4_pdas$pd.json 2> $O/f4_pdas$pd.log || { echo "f4 $pd failed"; tail -20 $O/f4_pdas$pd.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/f4_pdas$pd.json'))['f4'];print('PDAS=$pd', d['ms_per_step'], d['iter0_s'], d['roofline']['kernel_ms'], d['roofline']['polish_ms'], d['not_optimal_in_window'])"
done
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ -k "c1000 or uc_hub or teams or supernodal" > $O/pytest_gpu_r06_f4ab.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_gpu_r06_f4ab.log | tail -12
exit $rc
