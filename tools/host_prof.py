"""GPU diagnostic: where the wall time of one run_device_loop call goes on
the host (F2 bench window: farmer S, passes START+1 .. START+NIT in one
chunk): every batch method it calls timed with perf_counter, and the GPU
span (HIP events on the stream) beside the wall.

    python tools/host_prof.py S START NIT
"""
import os
import sys
import time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
import mpisppy_amd  # noqa: E402
mpisppy_amd.disable_tictoc_output()
from mpisppy_amd.opt.ph import PH  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402

S, START, NIT = (int(v) for v in sys.argv[1:4])
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 100000, "defaultPHrho": 1.0,
        "convthresh": -1, "verbose": False, "display_progress": False,
        "iter0_solver_options": {}, "iterk_solver_options": {}, "device_loop_graphs": False}
ph = PH(opts, [f"scen{i}" for i in range(S)], farmer.scenario_creator)
ph.PH_Prep()
ph.subproblem_creation()
ph.Iter0()
ph.run_device_loop(0, START, -1.0, chunk=NIT)
b = ph.batch
acc = {}
for name in ("loop_reset", "loop_enable", "loop_set_xbar", "loop_bind_pass", "xbar_accum", "loop_run",
             "loop_status", "loop_unbind_pass"):
    f = getattr(b, name)

    def w(*a, _f=f, _n=name, **k):
        t = time.perf_counter()
        r = _f(*a, **k)
        acc[_n] = acc.get(_n, 0.0) + time.perf_counter() - t
        return r
    setattr(b, name, w)
it = START
for rep in range(3):
    acc.clear()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    ph.run_device_loop(it, it + NIT, -1.0, chunk=NIT)
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e6
    it += NIT
    print(f"passes {it - NIT + 1}..{it}: wall {wall:.0f} us ({wall / NIT:.1f}/pass), stream span "
          f"{e0.elapsed_time(e1) * 1e3:.0f} us; host calls (us): " +
          ", ".join(f"{k} {v * 1e6:.0f}" for k, v in acc.items()), flush=True)
