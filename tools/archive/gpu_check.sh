#!/bin/bash
# F3 graph-replay repro, parity tests, one short bench line with the F3 companion
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/repro_f3.py 10000 100 1 3 > gpurun_out/repro_f3.log 2>&1 || { echo "F3 repro FAILED"; grep -v "^frame" gpurun_out/repro_f3.log | tail -6; exit 1; }
echo "F3 repro ok"; tail -2 gpurun_out/repro_f3.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --tol-run 0 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo "bench failed"; tail -30 gpurun_out/bench_quick.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_quick.json'));print(d['ms_per_step'], d['value'], {k:v['ms'] for k,v in d['roofline']['kernels'].items()}, d['hbm_config']['ms_per_step'])"
