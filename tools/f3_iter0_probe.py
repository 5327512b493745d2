"""GPU probe: farmer c=C Iter0 (cold LPs) on S scenarios; which scenarios stop
at the PDHG iteration limit, with their final KKT diagnostics, and the PDHG
step distribution.  Writes gpurun_out/f3_iter0.npz.

    python tools/f3_iter0_probe.py S C [max_iters]
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
MAXIT = int(sys.argv[3]) if len(sys.argv) > 3 else 200000
names = [f"scen{i}" for i in range(S)]
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 2, "defaultPHrho": 1.0, "convthresh": -1,
        "verbose": False, "display_progress": False,
        "iter0_solver_options": {"pdhg_max_iters": MAXIT}, "iterk_solver_options": {}}
ph = PH(opts, names, farmer.scenario_creator, scenario_creator_kwargs={"crops_multiplier": C})
ph.PH_Prep()
ph.subproblem_creation()
ph._create_solvers()
b = ph.batch
torch.cuda.synchronize()
t0 = time.time()
try:
    ph.Iter0()
except RuntimeError as e:
    print("Iter0 raised:", e)
torch.cuda.synchronize()
dt = time.time() - t0
st = b.status.cpu().numpy()
it = b.iters.cpu().numpy()
dg = b.diagnostics()
bad = np.nonzero(st != 0)[0]
print(f"Iter0 {dt:.2f}s  not optimal {bad.size}  iters p50 {np.percentile(it, 50):.0f} "
      f"p90 {np.percentile(it, 90):.0f} p99 {np.percentile(it, 99):.0f} max {it.max()}  "
      f"how counts {np.bincount(dg[:, 4].astype(int))}")
for s in bad[:40]:
    print("  scen", s, "iters", it[s], "ep %.2e ed %.2e eg %.2e r %.2e" % tuple(dg[s, :4]))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
X = b.x.view(b.n, b.S).cpu().numpy()
Y = b.y.view(-1, b.S).cpu().numpy()
np.savez(os.path.join(ROOT, "gpurun_out", f"f3_iter0_c{C}.npz"), bad=bad, iters=it, status=st,
         diag=dg, dbound=b.dbound.cpu().numpy(), pobj=b.pobj.cpu().numpy(),
         xbad=X[:, bad[:40]], ybad=Y[:, bad[:40]])
