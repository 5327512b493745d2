"""GPU diagnostic: phase clocks of the persistent device loop (loop_kernel,
ph_debug_prof slots 20-28) over NIT PH passes of farmer S (c=1), after START
warmup passes; also the same passes through the per-pass kernels
(PHGPU_PERSIST=0) for the wall time per pass.

    python tools/loop_prof.py S START NIT
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
from mpisppy_amd.examples import farmer  # noqa: E402

S, START, NIT = (int(v) for v in sys.argv[1:4])
names = [f"scen{i}" for i in range(S)]
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 100000, "defaultPHrho": 1.0,
        "convthresh": -1, "verbose": False, "display_progress": False,
        "iter0_solver_options": {}, "iterk_solver_options": {}, "device_loop_graphs": False}
ph = PH(opts, names, farmer.scenario_creator)
ph.PH_Prep()
ph.subproblem_creation()
ph.Iter0()
ph.run_device_loop(0, START, -1.0)
b = ph.batch
lib = b.lib
lib.ph_debug_prof.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
lib.ph_debug_prof.restype = ctypes.c_int32
it = START
for mode in ("1", "0", "1"):
    os.environ["PHGPU_PERSIST"] = mode
    out = np.zeros(32, dtype=np.int64)
    lib.ph_debug_prof(b.handle, 1, None)
    b.set_timing(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph.run_device_loop(it, it + NIT, -1.0, chunk=NIT)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / NIT * 1e6
    lk = b.loop_read_timing()
    b.set_timing(False)
    lib.ph_debug_prof(b.handle, 0, out.ctypes.data_as(ctypes.c_void_p))
    it += NIT
    st = b.loop_status()
    print(f"PHGPU_PERSIST={mode}: passes {it - NIT}..{it}: {dt:.1f} us per pass (wall), "
          f"misses {(st[3] - st[7]) / NIT:.1f} per pass, PDHG solves {st[3] - st[6] - st[7]}; "
          f"loop_kernel launches {lk[0]:.0f} ({lk[1] * 1e3 / NIT:.1f} us per pass inside them)", flush=True)
    if mode == "1":
        P = max(out[25], 1)
        nb = (S + 3) // 4 if S < 1024 else 256
        us = lambda t: t / 100.0 / P / nb  # 100 MHz ticks, per pass, per block
        print(f"  loop_kernel passes {out[25]}; per pass, block average: U {us(out[20]):.2f} "
              f"barrier-U {us(out[21]):.2f} combines {us(out[22]):.2f} S {us(out[23]):.2f} "
              f"barrier-S {us(out[24]):.2f} us; slowest block's S {out[26] / 100.0 / P:.2f} us; "
              f"polishes {out[28]} ({out[28] / P:.1f}/pass) at {out[27] / 100.0 / max(out[28], 1):.2f} us each",
              flush=True)
        print(f"  miss queue: {out[29] / P:.1f} queued/pass; drain {out[30] / 100.0 / P / (nb * 4):.2f} us per wave-pass; "
              f"slowest polish {out[31] / 100.0:.2f} us", flush=True)
