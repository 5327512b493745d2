#!/bin/bash
# parity tests, the polish phase profile, one short bench line
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u tools/polish_prof.py 10000 1 5 20 > gpurun_out/polprof.log 2>&1 || { echo "polprof failed"; tail -20 gpurun_out/polprof.log; exit 1; }
tail -6 gpurun_out/polprof.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --hbm-crops 0 --tol-run 0 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo "bench failed"; tail -30 gpurun_out/bench_quick.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_quick.json'));print(d['ms_per_step'], d['value'], {k:v['ms'] for k,v in d['roofline']['kernels'].items()})"
