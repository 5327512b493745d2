"""GPU diagnostic: PH ms/iteration of the device loop replayed as graphs vs
launched eagerly (the N>1 path launches eagerly around its collectives).

    python tools/loop_modes.py [S] [iters]
"""
import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
import mpisppy_amd
mpisppy_amd.disable_tictoc_output()
from mpisppy_amd.opt.ph import PH
from mpisppy_amd.examples import farmer

S = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
NIT = int(sys.argv[2]) if len(sys.argv) > 2 else 200
names = [f"scen{i}" for i in range(S)]
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 100000, "defaultPHrho": 1.0,
        "convthresh": -1, "verbose": False, "display_progress": False, "display_timing": False,
        "iter0_solver_options": {}, "iterk_solver_options": {}}
ph = PH(opts, names, farmer.scenario_creator, scenario_creator_kwargs={"crops_multiplier": 1})
ph.PH_Prep(); ph.subproblem_creation(); ph.Iter0()
it = 0
for graphs in (True, False, True, False):
    ph.PHoptions["device_loop_graphs"] = graphs
    ph.run_device_loop(it, it + 20, -1.0, chunk=20); it += 20  # warm / capture
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph.run_device_loop(it, it + NIT, -1.0, chunk=NIT if graphs else 16); it += NIT
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"graphs={graphs}: {dt / NIT * 1e3:.4f} ms/iteration", flush=True)
