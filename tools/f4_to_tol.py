"""GPU run: F4 (farmer crops_multiplier 1000, 1,000 scenarios) PH to
convergence, against the published EF objective -1.334838651e8
(paperruns/scripts/farmer/ef_1000_1000.out:182-183; BASELINE.md section 2,
F4 row).  Reports Iter0 (time, statuses, trivial bound), the iteration count
and conv, Eobj (ph_main's PH objective, phbase.py:279-312), the x-bar
objective (every scenario's objective at the common first stage, the
implementable solution's expected cost), post_solve_bound (phbase.py:753-801)
and the bracket post_solve_bound <= EF <= ... .

    python tools/f4_to_tol.py [S] [C] [convthresh] [limit] > out.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mpisppy_amd  # noqa: E402
mpisppy_amd.disable_tictoc_output()
from mpisppy_amd.opt.ph import PH  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
C = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
THRESH = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-4
LIMIT = int(sys.argv[4]) if len(sys.argv) > 4 else 20000
EF = -1.334838651e8 if (S, C) == (1000, 1000) else None
t00 = time.time()


def say(msg):
    print(f"[f4_to_tol {time.time() - t00:7.1f}] {msg}", file=sys.stderr, flush=True)


opts = {"solvername": "mi355x_pdhg", "PHIterLimit": LIMIT, "defaultPHrho": 1.0, "convthresh": THRESH,
        "verbose": False, "display_progress": False, "iter0_solver_options": {},
        "iterk_solver_options": {}}
ph = PH(opts, [f"scen{i}" for i in range(S)], farmer.scenario_creator,
        scenario_creator_kwargs={"crops_multiplier": C})
ph.PH_Prep()
ph.subproblem_creation()
ph._create_solvers()
torch.cuda.synchronize()
say(f"built n={ph.batch.n} m={ph.batch.m}")
t0 = time.perf_counter()
tb = ph.Iter0()
torch.cuda.synchronize()
t_iter0 = time.perf_counter() - t0
nonopt0 = int((ph.batch.status != 0).sum().item())
say(f"Iter0 {t_iter0:.2f} s, trivial bound {tb:.6f}, not optimal {nonopt0}")
it = 0
stop = 0
t1 = time.perf_counter()
while it < LIMIT and stop != 1:
    stop, it = ph.run_device_loop(it, min(it + 200, LIMIT), THRESH, chunk=50)
    conv = float(ph.conv_hist[it - 1].item()) if it > 0 else None
    say(f"PH iteration {it}: conv {conv:.3e} ({time.perf_counter() - t1:.1f} s)")
torch.cuda.synchronize()
t_loop = time.perf_counter() - t1
ph._PHIter = it
ph.conv = float(ph.conv_hist[it - 1].item())
eobj = ph.post_loops()
# the implementable first stage: every scenario at x-bar (the reference's
# xhat from the PH consensus), W and prox off
xb = ph.xbar.view(ph.K, ph.S_loc)[:, 0].cpu().numpy()
say("x-bar objective (xhat)")
ph._save_nonants()
ph._fix_nonants(xb)           # two-stage: node slot g = nonant slot k
kw = ph.solve_loop_launch(solver_options={"pdhg_max_iters": 100000}, dis_W=True, dis_prox=True)
ph.solve_loop_finish(kw)
xh_ok = bool((ph.batch.status == 0).all().item())
wd, pd = ph.W_disabled, ph.prox_disabled
ph._disable_W_and_prox()
xhat_obj = ph.Eobjective() if xh_ok else None
ph.W_disabled, ph.prox_disabled = wd, pd
ph._set_flags()
ph._restore_nonants()
say("post_solve_bound")
psb = ph.post_solve_bound()
out = {"scenarios": S, "crops_multiplier": C, "convthresh": THRESH,
       "iter0_s": round(t_iter0, 3), "iter0_not_optimal": nonopt0, "trivial_bound": tb,
       "ph_iterations": it, "stopped": "converged" if stop == 1 else "limit", "final_conv": ph.conv,
       "loop_seconds": round(t_loop, 2), "ms_per_iteration": round(t_loop / max(it, 1) * 1000, 2),
       "Eobj": eobj, "xhat_at_xbar": xhat_obj, "post_solve_bound": psb, "published_ef": EF}
if EF is not None:
    out["Eobj_rel_to_ef"] = (eobj - EF) / abs(EF)
    out["bracket_ok"] = bool(psb <= EF + 1e-9 * abs(EF) and tb <= EF)
    if xhat_obj is not None:
        out["xhat_rel_to_ef"] = (xhat_obj - EF) / abs(EF)
print(json.dumps(out))
