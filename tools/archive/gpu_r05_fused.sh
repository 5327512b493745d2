#!/bin/bash
# Round 5: the fused single-rank pass (finish_kernel): loop parity tests,
# phase stamps, F2 line (fused / PHGPU_FUSED=0), kernel-trace window
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "persistent or host_loop or farmer_ph or doc_farmer or 10k or iteration_limit or graphs or hub" > $O/pytest_r05_fused.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_r05_fused.log | tail -8
[ $rc -eq 0 ] || { grep -v "^frame" $O/pytest_r05_fused.log | tail -40; exit $rc; }
timeout -k 10 200 python -u tools/fin_prof.py 10000 5 > $O/fin_prof.txt 2>&1 || { tail -20 $O/fin_prof.txt; exit 1; }
grep pass $O/fin_prof.txt
B="--no-cpu-baseline --hbm-crops 0 --f4-scens 0 --sslp-scens 0 --uc-scens 0"
for mode in 1 0; do
  PHGPU_FUSED=$mode timeout -k 10 200 python -u bench.py $B > $O/f2_fused_$mode.json 2> $O/f2_fused_$mode.err || { echo "bench failed"; tail -20 $O/f2_fused_$mode.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/f2_fused_$mode.json'));print('fused=$mode', d['ms_per_step'], d['ph_to_tol']['seconds'], d['ph_to_tol']['ph_iterations'], d['ph_to_tol']['Eobj'], d['roofline']['kernel'], d['roofline']['kernel_ms'])"
done
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace -d $O/ktr3 -o ktr --output-format csv -- python3 $R/tools/host_prof.py 10000 5 20 > $O/host_prof_fused.txt 2>&1 || { tail -20 $O/host_prof_fused.txt; exit 1; }
grep passes $O/host_prof_fused.txt
python3 $R/tools/trace_window.py $O/ktr3/ktr_kernel_trace.csv 20 20
