#!/bin/bash
# Round 6: F4 with the team-size cap (PHGPU_BIG_TEAM_CAP 64 / default / 8)
# and with the 512-thread, two-per-CU polish build (libphgpu_p512.so copied
# over the library in this box's copy of the tree, last)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "c1000 or big_teams" > $O/pytest_team.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_team.log | tail -8
[ $rc -eq 0 ] || exit 1
f4() {  # tag, env...
  local T=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --tol-run 0 --no-cpu-baseline --only f4 --hbm-steps 5 --f4-bracket 0 > $O/f4_$T.json 2> $O/f4_$T.log || { echo "f4 $T failed"; tail -20 $O/f4_$T.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/f4_$T.json'))['f4'];print('$T', d['ms_per_step'], d['iter0_s'], d['roofline'].get('polish_ms'), d['roofline'].get('kernel_ms'))"
}
f4 cap64 PHGPU_BIG_TEAM_CAP=64 || exit 1
f4 capdef PHGPU_X=0 || exit 1
f4 cap8 PHGPU_BIG_TEAM_CAP=8 || exit 1
cp mpi-sppy_amd/mpisppy_amd/_lib/libphgpu_p512.so mpi-sppy_amd/mpisppy_amd/_lib/libphgpu.so
f4 p512 PHGPU_X=0 || exit 1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "c1000" > $O/pytest_p512.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_p512.log | tail -8
echo ALLDONE
