"""GPU probe: farmer c=C Iter0 LPs of the given scenario numbers only (the
F3 stragglers), with the PDHG iteration limit MAXIT; per scenario the
status, iterations and final KKT diagnostics.  Knobs come from the
library's PHGPU_* measurement environment variables.

    python tools/straggler_probe.py C MAXIT s1 s2 ...
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

C, MAXIT = int(sys.argv[1]), int(sys.argv[2])
ids = [int(v) for v in sys.argv[3:]]
names = [f"scen{i}" for i in ids]
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 2, "defaultPHrho": 1.0, "convthresh": -1,
        "verbose": False, "display_progress": False,
        "iter0_solver_options": {"pdhg_max_iters": MAXIT}, "iterk_solver_options": {}}
ph = PH(opts, names, farmer.scenario_creator, scenario_creator_kwargs={"crops_multiplier": C},
        all_nodenames=None)
ph.PH_Prep()
ph.subproblem_creation()
ph._create_solvers()
b = ph.batch
torch.cuda.synchronize()
t0 = time.time()
try:
    ph.Iter0()
except RuntimeError as e:
    print("Iter0 raised:", str(e)[:80])
torch.cuda.synchronize()
print(f"env {[(k, v) for k, v in os.environ.items() if k.startswith('PHGPU_')]}  {time.time() - t0:.2f}s")
st = b.status.cpu().numpy()
it = b.iters.cpu().numpy()
dg = b.diagnostics()
for s in range(len(ids)):
    print(f"  scen {ids[s]} status {st[s]} iters {it[s]} how {dg[s, 4]:.0f} "
          "ep %.2e ed %.2e eg %.2e r %.2e" % tuple(dg[s, :4]))
