#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no tol run / CPU baseline)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
TAG=${1:-prof}
shift
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$TAG -o run -- python3 bench.py --tol-run 0 --no-cpu-baseline "$@" > $O/$TAG.log 2>&1 || { echo "rocprof failed"; tail -30 $O/$TAG.log; exit 1; }
python3 - "$O/$TAG" <<'PY'
import csv, sys
d = sys.argv[1]
for r in csv.DictReader(open(d + "/run_kernel_stats.csv")):
    print(r["Name"][:70], r["Calls"], r["AverageNs"], r["Percentage"])
rows = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
pd = [i for i, r in enumerate(rows) if "pdhg_kernel" in r["Kernel_Name"]]
# gap analysis over the last 10 PH iterations
if len(pd) > 11:
    a, b = pd[-11], pd[-1]
    t0, t1 = int(rows[a]["End_Timestamp"]), int(rows[b]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a + 1:b + 1])
    print(f"last 10 iterations: wall {(t1 - t0) / 1e6 / 10:.4f} ms/iter, GPU busy {busy / 1e6 / 10:.4f} ms/iter, launches/iter {(b - a) / 10:.1f}")
PY
