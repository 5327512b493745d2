"""GPU diagnostic: phase clocks of the mid-size LDL' polish (ph_debug_prof
slots 9-15) over PH iterations of farmer S / c (eager device loop).

    python tools/mid_polish_prof.py S C START NIT      (C = 0: sslp_15_45 synthetic)
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
from mpisppy_amd.examples import farmer, sslp

S, C, START, NIT = (int(v) for v in sys.argv[1:5])
os.environ.setdefault("PHGPU_VERBOSE", "1")
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 100000, "defaultPHrho": 1.0,
        "convthresh": -1, "verbose": False, "display_progress": False,
        "iter0_solver_options": {}, "iterk_solver_options": {}, "device_loop_graphs": False}
if C == 0:
    ph = PH(opts, sslp.scenario_names(S), sslp.scenario_creator,
            scenario_creator_kwargs={"instance": "sslp_15_45_synthetic"})
else:
    ph = PH(opts, [f"scen{i}" for i in range(S)], farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": C})
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
t = b.read_timing_full()
lib.ph_debug_prof(b.handle, 0, out.ctypes.data_as(ctypes.c_void_p))
us = lambda v: v / 100.0  # 100 MHz ticks -> us (summed over blocks)
npol = max(out[9], 1)
st = b.loop_status()  # (counters since run_device_loop's reset: these NIT passes)
steps = int(st[4])
grid = 0
print(f"PDHG steps over the {NIT} passes: {steps} (last pass max {int(b.iters.max().item())}); "
      f"mid_kernel ms per 1000 steps: {t[5] / max(steps, 1) * 1000:.3f}")
print(f"iters {START}..{START+NIT}: mid_kernel {t[4]} launches {t[5]/max(t[4],1):.3f} ms avg, "
      f"mid_polish {t[6]} launches {t[7]/max(t[6],1):.3f} ms avg")
print(f"polishes {out[9]} ({out[9]/NIT:.0f}/iter), rounds {out[10]}, refinement solves {out[11]}, "
      f"accepted {out[12]} (in the first round {out[0]})")
print(f"per polish (block-us): setup {us(out[15] + out[27])/npol:.1f} (scatter {us(out[27])/npol:.1f}) "
      f"factor {us(out[13])/npol:.1f} solves {us(out[14])/npol:.1f} check {us(out[25])/npol:.1f} "
      f"PDAS {us(out[26])/npol:.1f}")
print(f"factors reused from the cache {out[28]} (of {out[10]} rounds)")
print(f"rounds with a pinned row {out[5]}; exits: accepted {out[12]}, set repeats {out[1]}, non-finite {out[2]}, round limit {out[3]}; "
      f"failed checks: refinement short {out[4]}, ep {out[6]}, ed {out[7]}, eg {out[8]}")
print(f"set repeats failing only the gap {out[20]}, rounds with a slack pinned row {out[21]}")
print(f"factorisations with a pivot held to its bound {out[16]}; non-finite: rhs {out[17]}, "
      f"refinement solve {out[18]}, check only {out[19]}")
nsc = max(out[30], 1)
print(f"PDHG phases: scenarios {out[30]}, steps {out[29]}; block-us per scenario: setup {us(out[22])/nsc:.1f} "
      f"end {us(out[31])/nsc:.1f}; per step: {us(out[23])/max(out[29],1):.2f} (+ checks {us(out[24])/max(out[29],1):.2f})")
