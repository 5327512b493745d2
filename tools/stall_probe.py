"""GPU probe: Iter0 of farmer S/C; per-scenario PDHG diagnostics of the
scenarios that stopped at the iteration limit.

    python tools/stall_probe.py S C [max_iters]
"""
import os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
import mpisppy_amd
mpisppy_amd.disable_tictoc_output()
from mpisppy_amd.opt.ph import PH
from mpisppy_amd.examples import farmer

S, C = int(sys.argv[1]), int(sys.argv[2])
mi = int(sys.argv[3]) if len(sys.argv) > 3 else 200000
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 1, "defaultPHrho": 1.0, "convthresh": -1,
        "verbose": False, "display_progress": False,
        "iter0_solver_options": {"pdhg_max_iters": mi}, "iterk_solver_options": {}}
names = [f"scen{i}" for i in range(S)]
ph = PH(opts, names, farmer.scenario_creator, scenario_creator_kwargs={"crops_multiplier": C})
ph.PH_Prep(); ph.subproblem_creation(); ph._create_solvers()
t = time.time(); tb = ph.Iter0(); torch.cuda.synchronize()
print(f"Iter0 {time.time()-t:.2f}s tb {tb:.8g}")
st = ph.batch.status.cpu().numpy(); it = ph.batch.iters.cpu().numpy()
dg = ph.batch.diagnostics()
bad = np.nonzero(st != 0)[0]
print("iters pct 50/90/99/max", np.percentile(it, [50, 90, 99]), it.max(), "not optimal", bad.size)
for s in bad[:12]:
    print(f"  scen{s}: iters {it[s]} ep {dg[s,0]:.2e} ed {dg[s,1]:.2e} eg {dg[s,2]:.2e} r {dg[s,3]:.2e}")
om = ph.batch.omega.cpu().numpy()
print("omega of bad:", om[bad[:12]])
