"""GPU probe of a PH workload: Iter0 time, then NIT PH iterations through the
device loop with per-kernel event timing, PDHG steps per solve and the
PDHG kernel's algorithmic bandwidth (SURVEY 8(d) B_it per step).

    python tools/workload_probe.py farmer S C NIT
    python tools/workload_probe.py sslp S 0 NIT        (sslp_15_45_synthetic)
"""
import os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
import mpisppy_amd
mpisppy_amd.disable_tictoc_output()
from mpisppy_amd.opt.ph import PH

wl, S, C, NIT = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
opts = {"solvername": "mi355x_pdhg", "PHIterLimit": 100000, "defaultPHrho": 1.0,
        "convthresh": -1, "verbose": False, "display_progress": False,
        "iter0_solver_options": {}, "iterk_solver_options": {}}
if wl == "farmer":
    from mpisppy_amd.examples import farmer as ex
    names = [f"scen{i}" for i in range(S)]
    kw = {"crops_multiplier": C}
else:
    from mpisppy_amd.examples import sslp as ex
    names = ex.scenario_names(S)
    kw = {"instance": "sslp_15_45_synthetic"}
t = time.time()
ph = PH(opts, names, ex.scenario_creator, scenario_creator_kwargs=kw)
ph.PH_Prep(); ph.subproblem_creation(); ph._create_solvers()
torch.cuda.synchronize()
print(f"{wl} S={S} C={C}: n={ph.batch.n} m={ph.batch.m} nnz={ph.batch.nnz} K={ph.K}; setup {time.time()-t:.1f}s", flush=True)
b = ph.batch
b.set_timing(True)
t = time.time(); tb = ph.Iter0(); torch.cuda.synchronize(); t0 = time.time() - t
n_t, as_ms, po_ms, pd_ms = b.read_timing()
s = b.summary()
print(f"Iter0: {t0*1e3:.1f} ms wall, pdhg kernel {pd_ms:.1f} ms, PDHG steps/solve {s[1]/S:.0f} (max {s[2]}), polished {s[3]}, tb {tb:.6g}", flush=True)
nnz, n, m = b.nnz, b.n, b.m
bit = 8 * (2 * nnz + 7 * n + 5 * m)
print(f"  Iter0 PDHG algorithmic {s[1]*bit/(pd_ms/1e3)/1e9:.0f} GB/s (B_it={bit} B/scenario-step)", flush=True)
b.set_timing(False)
ph.PHoptions["device_loop_graphs"] = False
b.set_timing(True)
t = time.time()
ph.run_device_loop(0, NIT, -1.0, chunk=NIT)
torch.cuda.synchronize(); dt = time.time() - t
n_t, as_ms, po_ms, pd_ms = b.read_timing()
st = b.loop_status()
print(f"{NIT} PH iterations: {dt/NIT*1e3:.2f} ms/iter wall (eager), kernels/iter: active_set {as_ms/n_t:.3f} polish {po_ms/n_t:.3f} pdhg {pd_ms/n_t:.3f} ms", flush=True)
print(f"  PDHG steps/solve {st[4]/max(st[3],1):.1f} (max {st[5]}), polished {st[6]}, cached {st[7]} of {st[3]} solves", flush=True)
if pd_ms > 0:
    print(f"  PDHG algorithmic {st[4]*bit/(pd_ms/1e3)/1e9:.0f} GB/s", flush=True)
