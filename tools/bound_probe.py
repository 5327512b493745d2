"""GPU probe: farmer (c=C, S scenarios) PH to convthresh, then
post_solve_bound at the given bound tolerances; per tolerance the count of
non-optimal bound solves, their KKT diagnostics and the bound.

    python tools/bound_probe.py S C [tol ...]
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
import mpisppy_amd  # noqa: E402
mpisppy_amd.disable_tictoc_output()
from mpisppy_amd.opt.ph import PH  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402

S, C = int(sys.argv[1]), int(sys.argv[2])
tols = [float(t) for t in sys.argv[3:]] or [1e-9, 1e-12]
names = [f"scen{i}" for i in range(S)]
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 60000, "defaultPHrho": 1.0, "convthresh": 1e-6,
        "verbose": False, "display_progress": False,
        "iter0_solver_options": {}, "iterk_solver_options": {}}
ph = PH(opts, names, farmer.scenario_creator, scenario_creator_kwargs={"crops_multiplier": C})
t0 = time.time()
conv, eobj, tb = ph.ph_main()
print(f"PH iters {ph._PHIter} conv {conv:.3e} eobj {eobj:.9f} tb {tb:.6f} ({time.time() - t0:.1f}s)")
b = ph.batch
for tol in tols:
    t0 = time.time()
    lb = ph.post_solve_bound(solver_options={"pdhg_tol": tol})
    torch.cuda.synchronize()
    st = b.status.cpu().numpy()
    it = b.iters.cpu().numpy()
    dg = b.diagnostics()
    bad = np.nonzero(st != 0)[0]
    print(f"tol {tol:.0e}: bound {lb:.9f} ({time.time() - t0:.2f}s) not optimal {bad.size} "
          f"how {np.bincount(dg[:, 4].astype(int) + 1)} iters p50 {np.percentile(it, 50):.0f} max {it.max()}")
    for s in bad[:12]:
        print("  scen", s, "iters", it[s], "ep %.2e ed %.2e eg %.2e r %.2e" % tuple(dg[s, :4]))
