#!/bin/bash
# The default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; tail -30 $O/bench_default.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/bench_default.json"))
print("F2", d["ms_per_step"], d["value"], d["ph_to_tol"]["seconds"], d["roofline"]["kernel"], d["roofline"]["frac"])
for k in ("hbm_config", "f4_config", "sslp_config"):
    c = d.get(k) or {}
    print(k, c.get("ms_per_step"), c.get("value"), c.get("iter0_s"), (c.get("roofline") or {}).get("frac"))
u = d.get("uc_config") or {}
print("uc", u.get("iter0_s"), u.get("ms_per_ph_iteration"))
PY
