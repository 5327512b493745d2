#!/bin/bash
# Round 5: cooperative launches + bundled xhat: the new tests, the teams /
# persistent / hub tests, the host's CPU share, a quick F2 loop timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
{ echo "nproc $(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c "import os;print('affinity',len(os.sched_getaffinity(0)))"; lscpu | grep -E "^CPU\(s\)|Thread|Core|Socket|Model name"; } > $O/host_cpu.txt 2>&1
cat $O/host_cpu.txt
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "bundled or async_spokes or spin_the_wheel or persistent or teams or xhat or c1000" > $O/pytest_r05_coop.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_r05_coop.log | tail -30
[ $rc -eq 0 ] || { tail -60 $O/pytest_r05_coop.log; exit $rc; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --hbm-crops 0 --sslp-scens 0 --f4-scens 0 --uc-scens 0 > $O/bench_r05_coop.json 2> $O/bench_r05_coop.err || { echo "bench failed"; tail -30 $O/bench_r05_coop.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_r05_coop.json'));print(d['ms_per_step'], d['ph_to_tol'])"
