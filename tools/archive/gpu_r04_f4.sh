#!/bin/bash
# Round 4: the new GPU tests (bundles, certificates incl. the big path, the
# F4 hard Iter0 LPs), the big polish's counters in Iter0 and 3 PH
# iterations, the F4 probe's timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "bundled or infeasible or unbounded or large_valued or hard_iter0 or c1000" --timeout 300 --timeout-method thread > $O/r04_pytest_new.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/r04_pytest_new.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc $rc"; tail -30 $O/r04_pytest_new.log; exit 1; }
timeout -k 10 300 python -u tools/big_polish_prof.py 1000 1000 3 > $O/r04_bigpol.txt 2>&1 || { echo "big polish prof failed"; tail -20 $O/r04_bigpol.txt; exit 1; }
cat $O/r04_bigpol.txt
timeout -k 10 300 python -u tools/f4_probe.py 1000 1000 3 > $O/r04_f4_probe.txt 2>&1 || { echo "f4 probe failed"; tail -20 $O/r04_f4_probe.txt; exit 1; }
cat $O/r04_f4_probe.txt
