"""Generate tests/golden/*.json (TEST INFRASTRUCTURE; run on CPU, no GPU).

farmer_ef.json -- the extensive form of the reference farmer generator
(examples/farmer/farmer.py:24-161, crops_multiplier=1, p=1/S) solved by the
oracle's HiGHS EF (oracle/ef.py, restating sputils.py:168-383) at the
BASELINE sizes.  The farmer subproblems are LPs, so the PH fixed point is the
EF optimum: the GPU PH run on 10k scenarios is checked against this file
(a size-independent property: PH converges to the EF's first stage and
objective).  The reference itself (Pyomo + a commercial solver) cannot run in
this image; the S=1000 entry is re-derived by the CPU suite
(tests/test_oracle.py) so the file stays pinned to the oracle.

    python tests/golden/make_golden.py
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import models as om  # noqa: E402
from oracle.ef import solve_ef  # noqa: E402


def farmer_ef(S, c=1):
    scens = [om.farmer(f"scen{i}", c, num_scens=S) for i in range(S)]
    t0 = time.time()
    obj, xs = solve_ef(scens)
    idx = scens[0].nodes[0][2]  # ROOT nonants in scenario_tree.py:36 order
    return {"S": S, "crops_multiplier": c, "ef_obj": obj,
            "nonants": [float(xs[0][i]) for i in idx],
            "nonant_names": [scens[0].var_names[i] for i in idx],
            "solve_s": round(time.time() - t0, 2)}


def main():
    out = {"source": "oracle/ef.py (HiGHS simplex) on oracle/models.farmer; p = 1/S",
           "cases": [farmer_ef(1000), farmer_ef(10000)]}
    with open(os.path.join(HERE, "farmer_ef.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
