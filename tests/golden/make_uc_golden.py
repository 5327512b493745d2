"""Golden UC LP-relaxation values (test fixture generator): the oracle's
restatement of paperruns/larger_uc/ReferenceModel_OK.py (oracle/models.uc,
binaries relaxed to [0, 1]) solved by HiGHS simplex for Scenario1..3 of the
1000scenarios_wind set, and the extensive forms of Scenario1..2 and 1..3.  Parity is UNPINNED: no reference file holds UC LP
values; these pin the GPU path to the oracle restatement only.

    python tests/golden/make_uc_golden.py > tests/golden/uc_lp_values.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from oracle import models as om  # noqa: E402
from oracle.solve import _highs_solve  # noqa: E402
from oracle.ef import solve_ef  # noqa: E402

out = {"source": "oracle/models.uc + HiGHS simplex (tests/golden/make_uc_golden.py)",
       "scenario_set": "1000scenarios_wind", "values": {}, "nonants_first": {}}
for nm in ("Scenario1", "Scenario2", "Scenario3"):
    t = time.time()
    sc = om.uc(nm)
    st, x, _, _ = _highs_solve(sc.c, None, sc.A, sc.rl, sc.ru, sc.l, sc.u, time_limit=600)
    out["values"][nm] = float(sc.c @ x)
    k = np.asarray(sc.nonant_idx) if hasattr(sc, "nonant_idx") else None
    out["nonants_first"][nm] = [float(v) for v in (x[k][:8] if k is not None else [])]
    print(nm, st, out["values"][nm], f"{time.time() - t:.1f}s", file=sys.stderr)
# the extensive forms of Scenario1..S (probability 1/S each): the optimum
# a hub's outer and inner bounds must bracket (sputils.create_EF restated)
out["ef"] = {}
for S in (2, 3):
    t = time.time()
    scens = [om.uc(f"Scenario{i + 1}") for i in range(S)]
    for sc in scens:
        sc.prob = 1.0 / S
    out["ef"][str(S)], _ = solve_ef(scens)
    print("EF", S, out["ef"][str(S)], f"{time.time() - t:.1f}s", file=sys.stderr)
print(json.dumps(out, indent=1))
