"""GPU diagnostic: the big path's polish exit counters (ph_debug_prof slots
of polish_big) in Iter0 and NIT PH iterations of farmer S / C, with the
first few scenarios' final KKT errors.

    python tools/big_polish_prof.py S C NIT
"""
import ctypes
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
import mpisppy_amd
mpisppy_amd.disable_tictoc_output()
from mpisppy_amd.opt.ph import PH
from mpisppy_amd.examples import farmer

S, C, NIT = (int(v) for v in sys.argv[1:4])
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 100000, "defaultPHrho": 1.0,
        "convthresh": -1, "verbose": False, "display_progress": False,
        "iter0_solver_options": {}, "iterk_solver_options": {}, "device_loop": False}
ph = PH(opts, [f"scen{i}" for i in range(S)], farmer.scenario_creator,
        scenario_creator_kwargs={"crops_multiplier": C})
ph.PH_Prep(); ph.subproblem_creation(); ph._create_solvers()
b = ph.batch
lib = b.lib
lib.ph_debug_prof.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
lib.ph_debug_prof.restype = ctypes.c_int32
out = np.zeros(32, dtype=np.int64)
names = {9: "polishes", 0: "accepted in the first round", 10: "rounds", 11: "refinement solves", 12: "accepted", 1: "nothing to change",
         2: "non-finite", 3: "round limit", 4: "refinement short", 6: "ep fails", 7: "ed fails",
         8: "eg fails", 20: "steps cut by the ratio test", 21: "full steps"}
def report(tag):
    lib.ph_debug_prof(b.handle, 0, out.ctypes.data_as(ctypes.c_void_p))
    d = b.diagnostics()
    st = b.status.cpu().numpy()
    print(tag, {v: int(out[k]) for k, v in names.items()}, "how", np.bincount(d[:, 4].astype(int), minlength=4),
          "not optimal", int((st != 0).sum()), flush=True)
    npol = max(int(out[9]), 1)
    if out[13] or out[14]:  # the prox-QP polish's phase clocks (100 MHz ticks)
        print("  block-us per polish: classification %.1f factor %.1f solves %.1f check %.1f "
              "re-classification %.1f" % tuple(out[k] / npol / 100.0 for k in (17, 13, 14, 15, 16)), flush=True)
    if out[22]:  # the first gap-only failure's decomposition (polish_big debug slots 23..29)
        g = out[23:30].copy().view(np.float64)
        print("  gap-only failure: free cols %.3e fixed cols %.3e active rows %.3e inactive rows %.3e "
              "pobj %.9e dobj %.9e eg %.3e" % tuple(g), flush=True)
lib.ph_debug_prof(b.handle, 1, None)
ph.Iter0()
report("Iter0")
import time  # noqa: E402
import torch  # noqa: E402
b.set_timing(True)
for k in range(NIT):
    lib.ph_debug_prof(b.handle, 1, None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph.Compute_Xbar(); ph.Update_W(False)
    ph.solve_loop(solver_options=ph.current_solver_options)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    it = b.iters.cpu().numpy()
    report(f"PH iteration {k + 1} ({dt * 1000:.1f} ms; PDHG steps max {it.max()}, scenarios with steps "
           f"{int((it > 0).sum())})")
