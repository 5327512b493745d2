#!/bin/bash
# Round 5: the persistent loop's miss queue: parity tests, phase clocks in the
# bench window (passes 5..25) and late, F2 line forced persistent / adaptive.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "persistent or host_loop or farmer_ph" > $O/pytest_r05_mq.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_r05_mq.log | tail -8
[ $rc -eq 0 ] || { grep -v "^frame" $O/pytest_r05_mq.log | tail -40; exit $rc; }
timeout -k 10 200 python -u tools/loop_prof.py 10000 5 20 > $O/loop_prof_mq_early.txt 2>&1 || { tail -20 $O/loop_prof_mq_early.txt; exit 1; }
grep -v amdgpu.ids $O/loop_prof_mq_early.txt
timeout -k 10 200 python -u tools/loop_prof.py 10000 50 200 > $O/loop_prof_mq_late.txt 2>&1 || { tail -20 $O/loop_prof_mq_late.txt; exit 1; }
grep -v amdgpu.ids $O/loop_prof_mq_late.txt
B="--no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0 --uc-scens 0"
for mode in 1 auto; do
  if [ $mode = auto ]; then unset PHGPU_PERSIST; else export PHGPU_PERSIST=$mode; fi
  timeout -k 10 200 python -u bench.py $B > $O/f2_mq_$mode.json 2> $O/f2_mq_$mode.err || { echo "bench failed"; tail -20 $O/f2_mq_$mode.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/f2_mq_$mode.json'));print('$mode', d['ms_per_step'], d['ph_to_tol']['seconds'], d['ph_to_tol']['ph_iterations'], d['ph_to_tol']['Eobj'], d['roofline']['kernel'], d['roofline']['kernel_ms'])"
done
