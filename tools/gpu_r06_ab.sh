#!/bin/bash
# Round 6: the captured-collective and UC cylinder tests, then F4 with and
# without the big path's scenario-slowest copies (PHGPU_BIG_TR), each under
# rocprofv3 --kernel-trace --stats (kernel means, scratch)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ -k "collective or uc_hub" > $O/pytest_gpu_r06_ab.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_gpu_r06_ab.log | tail -10
[ $rc -le 1 ] || exit $rc
for tr in 1 0; do
  PHGPU_BIG_TR=$tr timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/f4ab_$tr -o run -- python3 bench.py --tol-run 0 --no-cpu-baseline --only f4 --hbm-steps 5 --f4-bracket 0 > $O/f4ab_$tr.json 2> $O/f4ab_$tr.log || { echo "f4 ab $tr failed"; tail -20 $O/f4ab_$tr.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/f4ab_$tr.json'))['f4'];print('BIG_TR=$tr', d['ms_per_step'], d['iter0_s'], d['roofline']['kernel_ms'], d['roofline']['polish_ms'])"
  grep -E "big_polish|big_kernel|big_team|t_gather|t_scatter" $(find $O/f4ab_$tr -name '*kernel_stats.csv' | head -1) | cut -d, -f1-8
done
exit $rc
