"""GPU diagnostic: dump the warm-start state of the first scenarios after a
few PH iterations (polish off) for CPU-side analysis.

    python tools/dump_state.py S C NIT NSAVE OUT.npz
"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
import mpisppy_amd
mpisppy_amd.disable_tictoc_output()
from mpisppy_amd.opt.ph import PH
from mpisppy_amd.examples import farmer

S, C, NIT, NS, OUT = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
names = [f"scen{i}" for i in range(S)]
so = {"pdhg_polish": False}
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": NIT, "defaultPHrho": 1.0, "convthresh": -1,
        "verbose": False, "display_progress": False, "iter0_solver_options": dict(so),
        "iterk_solver_options": dict(so)}
ph = PH(opts, names, farmer.scenario_creator, scenario_creator_kwargs={"crops_multiplier": C})
ph.PH_Prep(); ph.subproblem_creation(); ph.Iter0()
for k in range(NIT):
    ph.Compute_Xbar(False); ph.Update_W(False); ph.conv = ph.convergence_diff()
    ph.solve_loop(solver_options=ph.current_solver_options)
ph.Compute_Xbar(False); ph.Update_W(False)
b = ph.batch
n, m, K = b.n, b.m, b.K
np.savez(OUT, x=b.x.view(n, S)[:, :NS].cpu().numpy(), y=b.y.view(m, S)[:, :NS].cpu().numpy(),
         W=ph.W.view(K, S)[:, :NS].cpu().numpy(), xbar=ph.xbar.view(K, S)[:, :NS].cpu().numpy(),
         rho=ph.rho.view(K, S)[:, :NS].cpu().numpy(), diag=b.diagnostics()[:NS])
print("saved", OUT)
