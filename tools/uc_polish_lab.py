"""CPU lab (development tool): the big path's LP polish (tools/lp_polish_lab.py's
restatements of PDHG and the ratio-test PDAS polish) on a UC LP relaxation
scenario (oracle.models.uc): from PDHG points at 1e-4 / 1e-6 / 1e-8, does the
polish finish, in how many rounds, and how far is its active set from the
exact one (HiGHS)?

    python tools/uc_polish_lab.py [Scenario1] [rounds]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from oracle import models as om  # noqa: E402
from oracle.solve import solve_scenario  # noqa: E402
import lp_polish_lab as lab  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "Scenario1"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 40
sc = om.uc(name)
t = time.time()
P = lab.Scaled(sc)
print(f"{name}: n={P.n} m={P.m} eta={P.eta:.4f} scaling {time.time() - t:.1f}s", flush=True)
t = time.time()
q = np.zeros(P.n)
xe, ye, feas = solve_scenario(sc.c, q, sc.A, sc.rl, sc.ru, sc.l, sc.u)
xes, yes_ = xe / P.dc, ye / P.dr
print(f"HiGHS: obj {sc.c @ xe:.10e} ({time.time() - t:.1f}s); scaled KKT {P.kkt(xes, yes_)[:3]}", flush=True)
x = np.zeros(P.n)
y = np.zeros(P.m)
om_ = None
steps = 0
for exit_err in (1e-4, 1e-5, 1e-6, 1e-7, 1e-8):
    t = time.time()
    x, y, it, err, om_ = lab.pdhg(P, x, y, exit_err, omega=om_, maxit=400000)
    steps += it
    print(f"PDHG to {exit_err:.0e}: {it} steps (total {steps}), err {err:.2e} ({time.time() - t:.1f}s); "
          f"|x-x*|inf {np.abs(x * P.dc - xe).max():.3e}", flush=True)
    t = time.time()
    res = lab.polish_rt(P, x.copy(), y.copy(), rounds=rounds, verbose=False)
    ok = res[0]
    print(f"  polish_rt: ok={ok} rounds {res[-1] if len(res) > 3 else '?'} ({time.time() - t:.1f}s)" +
          (f" obj {sc.c @ (res[1] * P.dc):.10e}" if ok else ""), flush=True)
    if ok:
        break
