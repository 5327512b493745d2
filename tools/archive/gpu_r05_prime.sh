#!/bin/bash
# Round 5: seeded hints for the first cached solve (Iter0): PH-to-tol
# breakdown with / without, the farmer parity tests, the F2 line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
for mode in 1 0; do
  PHGPU_PRIME=$mode timeout -k 10 200 python -u tools/tol_prof.py 10000 > $O/tol_prof_prime$mode.txt 2>&1 || { tail -20 $O/tol_prof_prime$mode.txt; exit 1; }
  echo "== PHGPU_PRIME=$mode"; grep -v amdgpu.ids $O/tol_prof_prime$mode.txt | grep "rep\|0\.\.25"
done
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "farmer or persistent or host_loop or 10k or iteration_limit or graphs or hub or xhat or bundle" > $O/pytest_r05_prime.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_r05_prime.log | tail -8
[ $rc -eq 0 ] || { grep -v "^frame" $O/pytest_r05_prime.log | tail -40; exit $rc; }
B="--no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0 --uc-scens 0"
timeout -k 10 200 python -u bench.py $B > $O/f2_prime.json 2> $O/f2_prime.err || { echo "bench failed"; tail -20 $O/f2_prime.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/f2_prime.json'));print(d['ms_per_step'], d['ph_to_tol'], d['ph_to_tol_sample']['seconds'])"
