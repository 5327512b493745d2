"""GPU diagnostic: where F2's PH-to-tolerance wall time goes (farmer S, c=1,
convthresh 1e-4): Iter0, then iterk_loop's device chunks (solve_log: wall
per chunk, solves, misses), by stretches of passes; PHGPU_PERSIST as set.

    python tools/tol_prof.py S [chunk]
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

S = int(sys.argv[1])
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 64
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 5000, "defaultPHrho": 1.0,
        "convthresh": 1e-4, "verbose": False, "display_progress": False,
        "iter0_solver_options": {}, "iterk_solver_options": {}, "device_loop_graphs": False,
        "device_loop_chunk": chunk}
for rep in range(2):
    ph = PH(opts, [f"scen{i}" for i in range(S)], farmer.scenario_creator)
    ph.PH_Prep()
    ph.subproblem_creation()
    ph._create_solvers()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph.Iter0()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ph.iterk_loop()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    log = ph.solve_log
    e0 = log[0]
    print(f"  Iter0 solve: {e0[0]} solves, {1e3 * e0[1]:.1f} ms, PDHG steps mean {e0[2]:.1f} max {e0[3]}, "
          f"polished+cached {e0[4]}", flush=True)
    print(f"rep {rep}: Iter0 {1e3 * (t1 - t0):.1f} ms, iterk_loop {1e3 * (t2 - t1):.1f} ms, "
          f"{ph._PHIter} iterations, {len(log)} log entries", flush=True)
    # by stretches of passes
    it = 0
    bands = [(0, 25), (25, 100), (100, 400), (400, 1000), (1000, 10 ** 9)]
    acc = {b: [0, 0.0, 0] for b in bands}
    for e in log:
        n_s, dt, _, _, npol = e
        passes = max(1, round(n_s / S))
        for b in bands:
            if b[0] <= it < b[1]:
                acc[b][0] += passes
                acc[b][1] += dt
                acc[b][2] += npol
        it += passes
    for b, (p, dt, npol) in acc.items():
        if p:
            print(f"  passes {b[0]}..{min(b[1], it)}: {p} passes, {1e3 * dt:.1f} ms, {1e6 * dt / p:.1f} us/pass, "
                  f"hits+polishes {npol / p / S:.4f} of scenarios", flush=True)
