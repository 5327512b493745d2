#!/bin/bash
# Round 5: instruction-fetch counters of polish_kernel / active_set_kernel /
# loop_kernel over F2's bench window (tools/polish_prof.py, per-pass kernels)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export PHGPU_PERSIST=${PERSIST:-0}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
  --kernel-include-regex "polish_kernel|active_set|loop_kernel" -d $O/pmc_ic -o ic --output-format csv -- python3 $R/tools/polish_prof.py 10000 1 5 20 > $O/pmc_ic.log 2>&1 || { tail -20 $O/pmc_ic.log; exit 1; }
tail -3 $O/pmc_ic.log
python3 - <<'PY'
import csv, glob, collections, os
O=os.environ.get("GRAFT_REPO_ROOT","/root/repo")+"/gpurun_out"
f=glob.glob(O+"/pmc_ic/**/*counter_collection.csv", recursive=True)
print(f)
agg=collections.defaultdict(lambda: collections.defaultdict(float)); nd=collections.Counter()
for fn in f:
    for r in csv.DictReader(open(fn)):
        k=r["Kernel_Name"][:60]; agg[k][r["Counter_Name"]]+=float(r["Counter_Value"]); nd[(k,r["Counter_Name"])]+=1
for k,v in agg.items():
    n=max(nd[(k,c)] for c in v)
    print(k, "dispatch-rows", n, {c: round(x/n,1) for c,x in sorted(v.items())})
PY
