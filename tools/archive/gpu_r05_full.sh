#!/bin/bash
# Round 5: the whole GPU suite, the default bench line (CPU baseline on the
# job's 16 CPUs), the CPU-baseline rank sweep, F4 PH to 1e-4 at HEAD.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ ${TESTK:+-k "$TESTK"} > $O/pytest_gpu_r05.log 2>&1; rc=$?
  grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu_r05.log | tail -20
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python -u bench.py > $O/bench_r05.json 2> $O/bench_r05.err || { echo "bench failed"; tail -30 $O/bench_r05.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_r05.json'));print(d['ms_per_step'], d['ph_to_tol']['seconds'], d['vs_cpu'], d['cpu_baseline']['cores'], d['cpu_baseline']['host'].get('cgroup_cpu_quota'), d['hbm_config']['ms_per_step'], d['f4_config']['ms_per_step'], d['sslp_config']['ms_per_step'])"
if [ "${SWEEP:-1}" = "1" ]; then
  timeout -k 10 400 python -u tools/cpu_ranks_sweep.py 30 16 32 64 128 > $O/cpu_ranks_sweep.json 2> $O/cpu_ranks_sweep.err || { echo "sweep failed"; tail -5 $O/cpu_ranks_sweep.err; }
  tail -4 $O/cpu_ranks_sweep.err
fi
timeout -k 10 300 python -u tools/f4_to_tol.py 1000 1000 1e-4 20000 > $O/f4_to_tol_1e-4.json 2> $O/f4_to_tol_1e-4.log || { echo "f4 failed"; tail -5 $O/f4_to_tol_1e-4.log; exit 1; }
cat $O/f4_to_tol_1e-4.json
