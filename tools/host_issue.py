"""GPU measurement: host issue time of one device-loop pass (ph_loop_pass:
one ctypes call launching update_w_conv + the solve's kernels) against the
GPU time of the pass, farmer S scenarios c=1, eager launches (no graph).

    python tools/host_issue.py [S] [PASSES]

Prints: host microseconds per pass spent issuing (the loop of
_device_iteration calls, which returns before the GPU finishes), and the
wall microseconds per pass of the whole chunk (GPU-bound when larger)."""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
import torch
import mpisppy_amd
mpisppy_amd.disable_tictoc_output()
from mpisppy_amd.opt.ph import PH
from mpisppy_amd.examples import farmer

S = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
N = int(sys.argv[2]) if len(sys.argv) > 2 else 200
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 100000, "defaultPHrho": 1.0,
        "convthresh": -1.0, "verbose": False, "display_progress": False,
        "iter0_solver_options": {}, "iterk_solver_options": {}, "device_loop_graphs": False}
ph = PH(opts, [f"scen{i}" for i in range(S)], farmer.scenario_creator)
ph.PH_Prep()
ph.subproblem_creation()
ph.Iter0()
ph.run_device_loop(0, 50, -1.0, chunk=50)  # warm the cache
b = ph.batch
kw = ph._solve_kwargs(ph.current_solver_options)
b.loop_reset(50, 50 + N, -1.0)
b.loop_enable(True)
b.loop_set_xbar(ph.prob_coeff, ph.slot_k, ph.slot_s0, ph.slot_s1, ph.xsums)
ph._bind_pass(kw)
b.xbar_accum(ph.prob_coeff, ph.slot_k, ph.slot_s0, ph.slot_s1, ph.xsums)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    ph._device_iteration(kw)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
st = b.loop_status()
b.loop_enable(False)
b.loop_unbind_pass()
print(f"S={S}: {N} passes, host issue {(t1 - t0) / N * 1e6:.1f} us/pass, "
      f"wall {(t2 - t0) / N * 1e6:.1f} us/pass, loop status {st[:2]}")
