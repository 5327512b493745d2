"""GPU diagnostic: per-solve PDHG iteration distribution and kernel time.

    python tools/iter_hist.py S C NIT
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

S, C, NIT = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
names = [f"scen{i}" for i in range(S)]
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": NIT, "defaultPHrho": 1.0, "convthresh": -1,
        "verbose": False, "display_progress": False, "iter0_solver_options": {},
        "iterk_solver_options": {}}
t0 = time.time()
ph = PH(opts, names, farmer.scenario_creator, scenario_creator_kwargs={"crops_multiplier": C})
ph.PH_Prep(); ph.subproblem_creation()
print(f"setup {time.time()-t0:.1f}s", flush=True)
b = ph.batch if hasattr(ph, "batch") else None


def report(tag, ms):
    it = ph.batch.iters.cpu().numpy()
    st = ph.batch.status.cpu().numpy()
    q = np.percentile(it, [50, 90, 99, 99.9])
    how = ph.batch.diagnostics()[:, 4].astype(int)
    hw = np.bincount(how, minlength=4)
    print(f"{tag}: kernel {ms:8.3f} ms  iters mean {it.mean():7.1f} p50 {q[0]:.0f} p90 {q[1]:.0f} "
          f"p99 {q[2]:.0f} p99.9 {q[3]:.0f} max {it.max()}  nonopt {(st != 0).sum()}  "
          f"sum/max {it.sum()/max(1,it.max()):.0f}  how(tol/warm-polish/polish/cache) {hw.tolist()}", flush=True)


e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); ph.Iter0(); e1.record(); torch.cuda.synchronize()
report("iter0(+bound)", e0.elapsed_time(e1))
for k in range(1, NIT + 1):
    ph.Compute_Xbar(False); ph.Update_W(False); ph.conv = ph.convergence_diff()
    e0.record()
    ph.batch.solve(ph.W, ph.rho, ph.xbar, ph.w_on, ph.prox_on)
    e1.record(); torch.cuda.synchronize()
    report(f"ph{k:3d}", e0.elapsed_time(e1))
