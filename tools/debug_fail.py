# GPU debug: find scenarios that hit the PDHG iteration limit and dump them
import sys, os, numpy as np, torch
sys.path.insert(0, "mpi-sppy_amd")
import mpisppy_amd; mpisppy_amd.disable_tictoc_output()
from mpisppy_amd.opt.ph import PH
from mpisppy_amd.examples import farmer
S = int(sys.argv[1]); NIT = int(sys.argv[2]); MAXIT = int(sys.argv[3])
names = [f"scen{i}" for i in range(S)]
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": NIT, "defaultPHrho": 1.0, "convthresh": -1,
        "verbose": False, "display_progress": False, "iter0_solver_options": {"pdhg_max_iters": MAXIT},
        "iterk_solver_options": {"pdhg_max_iters": MAXIT}}
ph = PH(opts, names, farmer.scenario_creator)
ph.PH_Prep(); ph.Iter0()
b = ph.batch
def snap():
    return dict(x=b.x.cpu().numpy().copy(), y=b.y.cpu().numpy().copy(), om=b.omega.cpu().numpy().copy())
for k in range(1, NIT + 1):
    ph.Compute_Xbar(False); ph.Update_W(False); ph.conv = ph.convergence_diff()
    pre = snap(); W = ph.W.cpu().numpy().copy(); xb = ph.xbar.cpu().numpy().copy()
    ph.solve_loop(solver_options=ph.current_solver_options)
    st = b.status.cpu().numpy(); it = b.iters.cpu().numpy(); dg = b.diagnostics()
    bad = np.nonzero(st != 0)[0]
    print(k, "conv", ph.conv, "fails", len(bad), "iters mean", it.mean(), "max", it.max(), flush=True)
    if len(bad):
        for s in bad[:5]:
            print("   scen", s, "diag", dg[s])
        np.savez(f"gpurun_out/fail_it{k}.npz", bad=bad, W=W, xbar=xb, x0=pre["x"], y0=pre["y"], om0=pre["om"],
                 diag=dg, iters=it, x=b.x.cpu().numpy(), S=S)
        break
