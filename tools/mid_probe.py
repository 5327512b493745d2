"""GPU probe of the mid-size path (scenarios larger than one wave): PH on
farmer c in {3, 10, 100} and sslp_15_45_5 against the oracle; then the
F3 workload (farmer c=100, 10k scenarios): Iter0 and PH iteration times.

    python tools/mid_probe.py [quick]
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
import mpisppy_amd  # noqa: E402
mpisppy_amd.disable_tictoc_output()
from mpisppy_amd.opt.ph import PH  # noqa: E402
from mpisppy_amd.examples import farmer, sslp  # noqa: E402
from oracle import models as om  # noqa: E402
from oracle.ph_oracle import OraclePH  # noqa: E402


def opts(**kw):
    o = {"solvername": "mi355x_pdhg", "PHIterLimit": 10, "defaultPHrho": 1.0, "convthresh": 1e-7,
         "verbose": False, "display_progress": False, "display_timing": False,
         "iter0_solver_options": {}, "iterk_solver_options": {}}
    o.update(kw)
    return o


def rel(a, b):
    a = np.asarray(a, float)
    b = np.asarray(b, float)
    return float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b))))


def compare(tag, ph, orc, res, ores):
    conv, eobj, tb = res
    oc, oe, ot = ores
    xb = ph.xbar.view(ph.K, ph.S_loc).cpu().numpy()[:, 0]
    W = ph.W.view(ph.K, ph.S_loc).cpu().numpy().T
    b = ph.batch
    dg = b.diagnostics()
    print(f"{tag}: iters {ph._PHIter}/{orc.iters} tb {tb:.10g}/{ot:.10g} ({abs(tb-ot)/abs(ot):.1e}) "
          f"Eobj {eobj:.10g}/{oe:.10g} ({abs(eobj-oe)/abs(oe):.1e}) xbar {rel(xb, orc.xbar[0]):.1e} "
          f"W {rel(W, np.array(orc.W)):.1e} how {np.bincount(dg[:, 4].astype(int), minlength=4)} "
          f"solves {len(ph.solve_log)} mean pdhg it {np.mean([x[2] for x in ph.solve_log]):.1f}",
          flush=True)


def run_farmer(c, S, first, it=10):
    names = [f"scen{i}" for i in range(first, first + S)]
    o = opts(PHIterLimit=it, convthresh=1e-7)
    t = time.time()
    ph = PH(dict(o), names, farmer.scenario_creator, scenario_creator_kwargs={"crops_multiplier": c})
    res = ph.ph_main()
    dt = time.time() - t
    orc = OraclePH(dict(o), [om.farmer(n, c) for n in names])
    ores = orc.ph_main()
    compare(f"farmer c={c} S={S} ({dt:.1f}s)", ph, orc, res, ores)


def run_sslp():
    names = sslp.scenario_names(5)
    o = opts(PHIterLimit=10, convthresh=1e-7)
    ph = PH(dict(o), names, sslp.scenario_creator,
            scenario_creator_kwargs={"data_dir": "data/sslp_15_45_5/scenariodata"})
    ph.PH_Prep()
    ph.subproblem_creation()
    tb = ph.Iter0()
    orc = OraclePH(dict(o), [om.sslp(n, "sslp_15_45_5") for n in names])
    ot = orc.Iter0()
    dg = ph.batch.diagnostics()
    print(f"sslp Iter0 tb {tb:.10g}/{ot:.10g} ({abs(tb-ot)/abs(ot):.1e}) status "
          f"{np.bincount(ph.batch.status.cpu().numpy())} how {np.bincount(dg[:, 4].astype(int))} "
          f"iters {ph.batch.iters.cpu().numpy()}", flush=True)


def run_f3(S=10000, c=100, nit=5):
    names = [f"scen{i}" for i in range(S)]
    o = opts(PHIterLimit=100000, convthresh=-1.0)
    ph = PH(dict(o), names, farmer.scenario_creator, scenario_creator_kwargs={"crops_multiplier": c})
    ph.PH_Prep()
    ph.subproblem_creation()
    ph._create_solvers()
    b = ph.batch
    torch.cuda.synchronize()
    t = time.time()
    try:
        ph.Iter0()
    except RuntimeError as e:
        print("Iter0 raised:", e)
    torch.cuda.synchronize()
    t0 = time.time() - t
    st = b.status.cpu().numpy()
    it = b.iters.cpu().numpy()
    dg = b.diagnostics()
    print(f"F3 Iter0 {t0:.3f}s status {np.bincount(st)} how {np.bincount(dg[:, 4].astype(int))} "
          f"pdhg it p50 {np.percentile(it, 50):.0f} p99 {np.percentile(it, 99):.0f} max {it.max()}",
          flush=True)
    import ctypes
    lib = b.lib
    lib.ph_debug_prof.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
    lib.ph_debug_prof.restype = ctypes.c_int32
    prof = np.zeros(32, dtype=np.int64)
    for k in range(nit):
        lib.ph_debug_prof(b.handle, 1, None)
        torch.cuda.synchronize()
        t = time.time()
        ph.Compute_Xbar()
        ph.Update_W(False)
        ph.solve_loop(solver_options={})
        torch.cuda.synchronize()
        dt = time.time() - t
        st = b.status.cpu().numpy()
        it = b.iters.cpu().numpy()
        dg = b.diagnostics()
        lib.ph_debug_prof(b.handle, 1, prof.ctypes.data_as(ctypes.c_void_p))
        npol = max(prof[9], 1)
        print(f"F3 PH it {k+1}: {dt*1000:.1f} ms status {np.bincount(st)} how "
              f"{np.bincount(dg[:, 4].astype(int), minlength=3)} pdhg it mean {it.mean():.1f} max {it.max()}"
              f" | polish {prof[9]} rounds/pol {prof[10]/npol:.2f} refine/pol {prof[11]/npol:.2f} ok {prof[12]}"
              f" us/pol: build {prof[15]/npol/100:.1f} factor {prof[13]/npol/100:.1f} solve {prof[14]/npol/100:.1f}",
              flush=True)


if __name__ == "__main__":
    quick = len(sys.argv) > 1 and sys.argv[1] == "quick"
    run_farmer(3, 12, 3)
    run_farmer(10, 12, 3)
    run_sslp()
    run_farmer(100, 12, 3, it=6)
    if not quick:
        run_f3()
