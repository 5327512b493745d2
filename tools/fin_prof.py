"""GPU diagnostic: finish_kernel's phase stamps (ph_debug_prof slots 16-19,
29-31) over one pass of farmer S after START passes (per-pass kernels).

    python tools/fin_prof.py S START
"""
import ctypes
import os
import sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
import mpisppy_amd  # noqa: E402
mpisppy_amd.disable_tictoc_output()
from mpisppy_amd.opt.ph import PH  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402

os.environ["PHGPU_PERSIST"] = "0"
S, START = (int(v) for v in sys.argv[1:3])
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 100000, "defaultPHrho": 1.0,
        "convthresh": -1, "verbose": False, "display_progress": False,
        "iter0_solver_options": {}, "iterk_solver_options": {}, "device_loop_graphs": False}
ph = PH(opts, [f"scen{i}" for i in range(S)], farmer.scenario_creator)
ph.PH_Prep()
ph.subproblem_creation()
ph.Iter0()
ph.run_device_loop(0, START, -1.0, chunk=START)
b = ph.batch
lib = b.lib
lib.ph_debug_prof.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
lib.ph_debug_prof.restype = ctypes.c_int32
it = START
for rep in range(4):
    out = np.zeros(32, dtype=np.uint64)
    lib.ph_debug_prof(b.handle, 1, None)
    ph.run_device_loop(it, it + 1, -1.0, chunk=1)  # (one pass: its finish_kernel without the next update)
    lib.ph_debug_prof(b.handle, 0, out.ctypes.data_as(ctypes.c_void_p))
    it += 1
    t0 = int(out[16])
    us = lambda v: (int(v) - t0) / 100.0 if int(v) else float("nan")
    print(f"pass {it}: (us from block 0's start) polish end {us(out[17]):.1f} "
          f"tail end {us(out[18]):.1f} sums ready {us(out[19]):.1f} update end {us(out[29]):.1f}; "
          f"working polish blocks {int(out[30])}, longest release fence {int(out[31]) / 100.0:.2f} us", flush=True)
