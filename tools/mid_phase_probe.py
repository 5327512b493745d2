"""GPU probe: the mid-size path's phase launches one by one (ph_debug_phase_times)
over NIT single PH passes of sslp_15_45 synthetic (or farmer c=C) with S
scenarios, after W warmup passes: per launch kind and ms, the phase list
counts, and the PDHG step distribution of the solve (which scenarios hold
the grid).

    python tools/mid_phase_probe.py sslp|farmerC S W NIT
"""
import ctypes
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

model, S, W, NIT = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 100000, "defaultPHrho": 1.0,
        "convthresh": -1, "verbose": False, "display_progress": False,
        "iter0_solver_options": {}, "iterk_solver_options": {}, "device_loop_graphs": False}
if model == "sslp":
    from mpisppy_amd.examples import sslp as ex
    ph = PH(opts, ex.scenario_names(S), ex.scenario_creator,
            scenario_creator_kwargs={"instance": "sslp_15_45_synthetic"})
else:
    from mpisppy_amd.examples import farmer
    ph = PH(opts, [f"scen{i}" for i in range(S)], farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": int(model[6:])})
ph.PH_Prep()
ph.subproblem_creation()
t0 = time.time()
ph.Iter0()
torch.cuda.synchronize()
b = ph.batch
print(f"Iter0 {time.time() - t0:.2f} s; n={b.n} m={b.m} nnz={b.nnz}", flush=True)
ph.run_device_loop(0, W, -1.0, chunk=1)
lib = b.lib
lib.ph_debug_phase_times.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
lib.ph_debug_phase_times.restype = ctypes.c_int32
lib.ph_debug_prof.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
lib.ph_debug_prof.restype = ctypes.c_int32
prof = np.zeros(64, dtype=np.int64)
it = W
for k in range(NIT):
    b.set_timing(True)
    lib.ph_debug_prof(b.handle, 1, None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph.run_device_loop(it, it + 1, -1.0, chunk=1)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) * 1e3
    it += 1
    out = np.zeros(64, dtype=np.float64)
    ctr = np.zeros(16, dtype=np.int32)
    nk = lib.ph_debug_phase_times(b.handle, out.ctypes.data_as(ctypes.c_void_p), 32,
                                  ctr.ctypes.data_as(ctypes.c_void_p))
    n_t, as_ms, po_ms, pd_ms = b.read_timing()
    b.set_timing(False)
    lib.ph_debug_prof(b.handle, 1, prof.ctypes.data_as(ctypes.c_void_p))
    nst, nsc = max(int(prof[29]), 1), max(int(prof[30]), 1)
    # solve_mid's block clocks (100 MHz ticks): [22] setup [23] steps [24] checks [31] end
    prof_s = (f"mid PDHG: {nsc} scenario-phases, {nst} steps, us/step (block) steps "
              f"{prof[23] / nst / 100:.2f} checks {prof[24] / nst / 100:.2f}; us/scenario-phase setup "
              f"{prof[22] / nsc / 100:.1f} end {prof[31] / nsc / 100:.1f}")
    iters = b.iters.cpu().numpy()
    order = np.argsort(-iters)[:8]
    d = b.diagnostics()
    ph_s = " ".join(f"{'P' if out[2 * i] == 1 else 'D'}{out[2 * i + 1]:.2f}" for i in range(nk))
    print(f"pass {it}: {dt:.1f} ms wall; phases [{ph_s}] ms; lists {ctr[:7].tolist()}; "
          f"PDHG steps mean {iters.mean():.1f} max {iters.max()} >100: {(iters > 100).sum()} "
          f">500: {(iters > 500).sum()}; top {[(int(s), int(iters[s])) for s in order]}; "
          f"how {np.bincount(d[:, 4].astype(int), minlength=4).tolist()}; {prof_s}", flush=True)
