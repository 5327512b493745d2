#!/bin/bash
# Round 5: grouped active-set kernel (four scenarios per wave): parity tests,
# the F2 line with / without, the kernel-trace window
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "farmer or persistent or host_loop or 10k or iteration_limit or graphs or hub or xhat or bundle or hydro" > $O/pytest_r05_asg.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_r05_asg.log | tail -8
[ $rc -eq 0 ] || { grep -v "^frame" $O/pytest_r05_asg.log | tail -40; exit $rc; }
B="--no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0 --uc-scens 0"
for mode in 1 0 1; do
  PHGPU_AS_GROUPED=$mode timeout -k 10 200 python -u bench.py $B > $O/f2_asg_$mode.json 2> $O/f2_asg_$mode.err || { echo "bench failed"; tail -20 $O/f2_asg_$mode.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/f2_asg_$mode.json'));print('grouped=$mode', d['ms_per_step'], d['ph_to_tol']['seconds'], d['ph_to_tol']['ph_iterations'], d['ph_to_tol']['Eobj'], d['roofline']['kernels'])"
done
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace -d $O/ktr4 -o ktr --output-format csv -- python3 $R/tools/host_prof.py 10000 5 20 > $O/host_prof_asg.txt 2>&1 || { tail -20 $O/host_prof_asg.txt; exit 1; }
grep passes $O/host_prof_asg.txt
python3 $R/tools/trace_window.py $O/ktr4/ktr_kernel_trace.csv 20 20
