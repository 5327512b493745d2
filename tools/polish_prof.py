"""GPU diagnostic: phase clocks of pdhg_kernel's warm polish (ph_debug_prof)
over PH iterations of farmer S/C in eager device-loop mode.

    python tools/polish_prof.py S C START NIT
"""
import ctypes, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
import mpisppy_amd
mpisppy_amd.disable_tictoc_output()
from mpisppy_amd.opt.ph import PH
from mpisppy_amd.examples import farmer

S, C, START, NIT = (int(v) for v in sys.argv[1:5])
names = [f"scen{i}" for i in range(S)]
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 100000, "defaultPHrho": 1.0,
        "convthresh": -1, "verbose": False, "display_progress": False,
        "iter0_solver_options": {}, "iterk_solver_options": {}, "device_loop_graphs": False}
ph = PH(opts, names, farmer.scenario_creator, scenario_creator_kwargs={"crops_multiplier": C})
ph.PH_Prep(); ph.subproblem_creation(); ph.Iter0()
ph.run_device_loop(0, START, -1.0)
b = ph.batch
lib = b.lib
lib.ph_debug_prof.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
lib.ph_debug_prof.restype = ctypes.c_int32
out = np.zeros(32, dtype=np.int64)
lib.ph_debug_prof(b.handle, 1, None)
b.set_timing(True)
ph.run_device_loop(START, START + NIT, -1.0, chunk=NIT)
n_t, as_ms, po_ms, pd_ms = b.read_timing()
lib.ph_debug_prof(b.handle, 0, out.ctypes.data_as(ctypes.c_void_p))
st = b.loop_status()
npol = max(out[0], 1)
us = lambda t: t / 100.0  # 100 MHz ticks -> us
print(f"iters {START}..{START+NIT}: active_set {as_ms/max(n_t,1)*1e3:.1f} us, polish {po_ms/max(n_t,1)*1e3:.1f} us, pdhg {pd_ms/max(n_t,1)*1e3:.1f} us per solve")
npk = max(out[15], 1)
print(f"polish_kernel: accepted {out[15]} ({out[15]/NIT:.0f}/iter); per accepted: start {us(out[9])/npk:.2f} loads {us(out[10])/npk:.2f} build {us(out[11])/npk:.2f} GJ {us(out[12])/npk:.2f} check {us(out[13])/npk:.2f} store {us(out[14])/npk:.2f} us")
print(f"warm polishes {out[0]} ({out[0]/NIT:.0f}/iter): prologue {us(out[1])/npol:.2f} us, polish {us(out[2])/npol:.2f} us")
print(f"GJ solves {out[3]} ({out[3]/npol:.2f}/polish), GJ {us(out[4])/max(out[3],1):.2f} us each, cache store {us(out[5])/npol:.2f} us")
print(f"ok 1st attempt {out[6]}, ok 2nd {out[7]}, failed {out[8]}")
