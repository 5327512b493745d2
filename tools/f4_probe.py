"""GPU probe of the big path (farmer crops_multiplier C, S scenarios):
Iter0 time and statuses, the trivial bound (a lower bound of the EF; S=1000
C=1000: the published EF is -1.334838651e8,
paperruns/scripts/farmer/ef_1000_1000.out:183), then NIT PH iterations
through the device loop with per-launch timing and the big_kernel's
streaming rate (SURVEY 8(d) B_it per scenario-step).

    python tools/f4_probe.py S C NIT
"""
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

S, C, NIT = (int(v) for v in sys.argv[1:4])
t0 = time.time()
def say(m):
    print(f"[{time.time() - t0:7.1f}] {m}", flush=True)
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 100000, "defaultPHrho": 1.0,
        "convthresh": -1.0, "verbose": False, "display_progress": False,
        "iter0_solver_options": {}, "iterk_solver_options": {}, "device_loop_graphs": False}
ph = PH(opts, [f"scen{i}" for i in range(S)], farmer.scenario_creator,
        scenario_creator_kwargs={"crops_multiplier": C})
ph.PH_Prep()
ph.subproblem_creation()
ph._create_solvers()
b = ph.batch
torch.cuda.synchronize()
say(f"built: n={b.n} m={b.m} nnz={b.nnz}")
t = time.perf_counter()
tb = ph.Iter0()
torch.cuda.synchronize()
st = b.status.cpu().numpy()
it = b.iters.cpu().numpy()
say(f"Iter0 {time.perf_counter() - t:.3f} s: trivial bound {tb:.6f}, not optimal {(st != 0).sum()}, "
    f"PDHG steps mean {it.mean():.0f} max {it.max()}")
n, m, nnz = b.n, b.m, b.nnz
bit = 8 * (2 * nnz + 7 * n + 5 * m)
for k in range(NIT):
    b.set_timing(True)
    t = time.perf_counter()
    ph.run_device_loop(k, k + 1, -1.0, chunk=1)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    nt, _, _, _, nk, k_ms, np_, p_ms = b.read_timing_full()
    ls = b.loop_status()
    b.set_timing(False)
    steps = ls[4]
    gbs = steps * bit / (k_ms / 1000.0) / 1e9 if k_ms > 0 else 0.0
    say(f"PH iteration {k + 1}: {dt * 1000:.1f} ms; big_kernel {nk} launches {k_ms:.2f} ms, "
        f"polish {np_} launches {p_ms:.2f} ms; PDHG steps {steps} (mean {steps / S:.1f}, max {ls[5]}); "
        f"polished {ls[6]}; not optimal {ls[2]}; streaming {gbs:.0f} GB/s ({gbs / 8000:.3f} of 8 TB/s)")
