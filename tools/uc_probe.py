"""GPU probe of the UC LP relaxation (examples/uc.py, BASELINE config 4):
Iter0 of S scenarios through the big path (y in the workspace slice: m =
69,902 rows), its statuses / PDHG steps / time, the trivial bound against
the oracle's HiGHS LP values (first 3 scenarios), then NIT PH iterations
with the reference's rho setter (uc_funcs.py:94-112).

    python tools/uc_probe.py S NIT [max_iters] [tol]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mpisppy_amd  # noqa: E402
mpisppy_amd.disable_tictoc_output()
from mpisppy_amd.opt.ph import PH  # noqa: E402
from mpisppy_amd.examples import uc  # noqa: E402

S = int(sys.argv[1])
NIT = int(sys.argv[2])
MAXIT = int(sys.argv[3]) if len(sys.argv) > 3 else 200000
TOL = float(sys.argv[4]) if len(sys.argv) > 4 else 1e-9
t0 = time.time()


def say(m):
    print(f"[uc_probe {time.time() - t0:7.1f}] {m}", flush=True)


def _heartbeat():  # the solves block in one library call; keep the log moving
    while True:
        time.sleep(30)
        print(f"[uc_probe {time.time() - t0:7.1f}] ...", flush=True)


import threading  # noqa: E402
threading.Thread(target=_heartbeat, daemon=True).start()


opts = {"solvername": "mi355x_pdhg", "PHIterLimit": NIT, "defaultPHrho": 1.0, "convthresh": -1.0,
        "verbose": False, "display_progress": False,
        "iter0_solver_options": {"pdhg_max_iters": MAXIT, "pdhg_tol": TOL},
        "iterk_solver_options": {"pdhg_max_iters": MAXIT, "pdhg_tol": TOL}, "device_loop": False}
names = uc.all_scenario_names(S)
ph = PH(opts, names, uc.scenario_creator, rho_setter=uc.scenario_rhos)
ph.PH_Prep()
ph.subproblem_creation()
say("creating the batch (KKT symbolic analysis)")
ph._create_solvers()
b = ph.batch
torch.cuda.synchronize()
say(f"built n={b.n} m={b.m} nnz={b.nnz} K={b.K}")
b.set_timing(True)
import ctypes  # noqa: E402
_lib = b.lib
_lib.ph_debug_prof.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
_lib.ph_debug_prof.restype = ctypes.c_int32
_prof = np.zeros(64, dtype=np.int64)


def prof_reset():
    _lib.ph_debug_prof(b.handle, 1, None)


def prof_read(tag):
    _lib.ph_debug_prof(b.handle, 1, _prof.ctypes.data)
    p = _prof
    say(f"  {tag} polish counters: polishes {p[9]} rounds {p[10]} solves {p[11]} accepted {p[12]}; "
        f"no change {p[1]} non-finite {p[2]} round limit {p[3]} refine short {p[4]} fail ep/ed/eg {p[6]}/{p[7]}/{p[8]}")


prof_reset()
t = time.perf_counter()
tb = ph.Iter0()
torch.cuda.synchronize()
dt = time.perf_counter() - t
st = b.status.cpu().numpy()
it = b.iters.cpu().numpy()
d = b.diagnostics()
say(f"Iter0 {dt:.2f} s: trivial bound {tb:.6f}, statuses {np.bincount(st, minlength=4)}, PDHG steps mean "
    f"{it.mean():.0f} max {it.max()}, how {np.bincount(d[:, 4].astype(int), minlength=4)}; per scenario "
    f"{it.tolist()}")
print("  final errors of the first scenarios:", d[:3, :3], flush=True)
nt, _, _, _, nk, k_ms, np_, p_ms = b.read_timing_full()
say(f"  big_kernel {nk} launches {k_ms:.1f} ms, polish {np_} launches {p_ms:.1f} ms; "
    f"{k_ms / max(it.sum() / S, 1):.4f} ms per PDHG step (per scenario, in parallel)")
prof_read("Iter0")
if S <= 8:
    from oracle import models as om
    from oracle.solve import _highs_solve
    vals = []
    for nm in names[:3]:
        sc = om.uc(nm)
        stt, x, _, _ = _highs_solve(sc.c, None, sc.A, sc.rl, sc.ru, sc.l, sc.u, time_limit=120)
        vals.append(float(sc.c @ x))
    ob = (b.dbound.cpu().numpy() + b.const.cpu().numpy())[:3]
    say(f"oracle LP values {vals}; GPU outer bounds {ob.tolist()}; rel {(ob - vals) / np.abs(vals)}")
for k in range(NIT):
    prof_reset()
    t = time.perf_counter()
    ph.Compute_Xbar()
    ph.Update_W(False)
    ph.solve_loop(solver_options=ph.current_solver_options)
    torch.cuda.synchronize()
    st = b.status.cpu().numpy()
    it = b.iters.cpu().numpy()
    d = b.diagnostics()
    say(f"PH iteration {k + 1}: {1000 * (time.perf_counter() - t):.1f} ms, statuses {np.bincount(st, minlength=4)}, "
        f"PDHG steps mean {it.mean():.0f} max {it.max()}, how {np.bincount(d[:, 4].astype(int), minlength=4)}")
    nt, _, _, _, nk, k_ms, np_, p_ms = b.read_timing_full()
    say(f"  big_kernel {nk} launches {k_ms:.1f} ms, polish {np_} launches {p_ms:.1f} ms")
    prof_read(f"PH {k + 1}")
