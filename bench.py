#!/usr/bin/env python
"""Benchmark: farmer PH on MI355X -- scenario prox-QP solves/sec (+ PH wall-clock to tol).

A "step" is one PH iteration of the hot path over the whole scenario set:
Compute_Xbar -> Update_W -> convergence_diff (device kernels + RCCL allreduce)
-> solve_loop (the batched solve of every local scenario's prox-QP to 1e-9
relative KKT).  Steps run through the device-side PH loop (PHBase.
run_device_loop), replayed as HIP graphs on one GPU.

Scaling is weak: every rank holds --scens scenarios (10,000 by default, the
BASELINE config on one GPU), so N GPUs solve N x 10,000 scenarios per step;
scenarios are split over ranks as the reference does (contiguous slices).
The PH-to-tolerance run ("ph_to_tol") is always the 10,000-scenario instance
(strong: the same problem on N GPUs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scens S] [--crops C]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.  Input data are synthetic farmer instances
generated exactly as the reference's examples/farmer/farmer.py does.
"""
import argparse
import contextlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def farmer_dims(c):
    return 12 * c, 1 + 9 * c, 27 * c  # n, m, nnz per scenario


def bytes_per_pdhg_iter(c):
    """B_it/S = 8*(2*nnz + 7*n + 5*m) bytes per scenario per
    fused PDHG iteration (SpMV + SpMV^T values, x/g/q/l/u, y/rl/ru)."""
    n, m, nnz = farmer_dims(c)
    return 8 * (2 * nnz + 7 * n + 5 * m)


def solve_bytes_per_scenario(c):
    """HBM bytes one scenario solve must move at least: scaled matrix values
    (nnz), row/column scalings (m+n), c/l/u (3n), rl/ru (2m), the x/y warm
    start in and the solution out (2n+2m), W/rho/xbar (3K), step size,
    primal weight in/out, status/iters, pobj/dbound and diagnostics (13)."""
    n, m, nnz = farmer_dims(c)
    K = 3 * c
    return 8 * (nnz + (n + m) + 3 * n + 2 * m + 2 * (n + m) + 3 * K + 13)


_CPU_PROBS = None  # the sample's subproblems, inherited by forked workers


def _cpu_worker(arg):
    """Solve the sample's subproblems w, w+k, w+2k, ... cyclically until
    `min_seconds` have passed; (solves, seconds)."""
    from oracle.solve import _highs_solve
    w, k, min_seconds = arg
    mine = _CPU_PROBS[w::k]
    n = 0
    t0 = time.perf_counter()
    while True:
        for pr in mine:
            _highs_solve(*pr)
        n += len(mine)
        dt = time.perf_counter() - t0
        if dt >= min_seconds:
            return n, dt


def cpu_subproblem_rate(c, sample_scens, min_seconds=10.0, cores=16):
    """Oracle subproblem engine (HiGHS 1.8 from scipy) timed on this host on a
    bounded sample: the prox-QPs of one PH iteration (W and xbar from an
    oracle Iter0) for `sample_scens` farmer c=`c` scenarios, solved
    sequentially per process like the reference's solve_loop, each of
    `cores` forked processes cycling its share for `min_seconds`.  Runs
    before anything touches the GPU (the workers are forked)."""
    global _CPU_PROBS
    import multiprocessing as mp
    sys.path.insert(0, ROOT)
    from oracle import models as om
    from oracle.ph_oracle import OraclePH
    names = [f"scen{i}" for i in range(sample_scens)]
    scens = [om.farmer(nm, c) for nm in names]
    ph = OraclePH({"PHIterLimit": 1, "defaultPHrho": 1.0, "convthresh": 0.0}, scens)
    ph.Iter0()
    ph.Compute_Xbar()
    ph.Update_W()
    probs = []
    for s in range(len(scens)):
        g, q, _ = ph._terms(s, 1.0, 1.0)
        sc = scens[s]
        probs.append((g, q, sc.A, sc.rl, sc.ru, sc.l, sc.u))
    _CPU_PROBS = probs
    cores = max(1, min(cores, len(os.sched_getaffinity(0)), len(probs)))
    with mp.get_context("fork").Pool(cores) as pool:
        res = pool.map(_cpu_worker, [(w, cores, min_seconds) for w in range(cores)])
    nm = sum(r[0] for r in res)
    dtm = max(r[1] for r in res)
    return {"value": round(nm / dtm, 2), "unit": "solves/s", "cores": cores, "kind": "port",
            "sample": f"{len(probs)} distinct farmer c={c} PH prox-QPs of one PH iteration after "
                      f"Iter0 (HiGHS 1.8.0 QP via scipy, no polish), cycled on {cores} processes "
                      f"x {dtm:.1f} s ({nm} solves)"}


def cpu_baseline(c, scens, convthresh, cores=16, f3_crops=100, f3_sample=64, f3_seconds=8.0,
                 n1_iters=50):
    """the oracle PH (oracle/ph_dist.py: phbase.py's
    Iter0/iterk control flow, exact HiGHS + KKT-polish subproblem solves,
    Compute_Xbar/convergence_diff allreduces) on `cores` gloo ranks of this
    host, the same farmer instance and convthresh as the GPU's PH-to-tol
    run, at `scens` scenarios (a bounded sample of the 10k workload; the GPU
    runs the same size too, see ph_to_tol_sample).  value = subproblem
    solves / wall seconds of that run.  Plus a c=`f3_crops` subproblem-rate
    sample for the F3 companion config."""
    sys.path.insert(0, ROOT)
    from oracle import ph_dist
    cores = job_cpus() if cores <= 0 else max(1, min(cores, len(os.sched_getaffinity(0))))
    t0 = time.perf_counter()
    r = ph_dist.run(cores, scens, crops=c, rho=1.0, convthresh=convthresh)
    wall = time.perf_counter() - t0
    out = {"value": round(r["subproblem_solves"] / r["seconds_to_tol"], 2), "unit": "solves/s",
           "cores": cores, "kind": "port",
           "sample": f"oracle PH (oracle/ph_dist.py) on {cores} gloo ranks, farmer c={c}, "
                     f"{scens} scenarios, rho 1, convthresh {convthresh}: {r['iterations']} PH "
                     f"iterations, {r['subproblem_solves']} exact subproblem solves in "
                     f"{r['seconds_to_tol']:.2f} s (Iter0 {r['seconds_iter0']:.2f} s; "
                     f"{wall:.1f} s with rank start-up)",
           "ph_to_tol": {"seconds": round(r["seconds_to_tol"], 3), "ph_iterations": r["iterations"],
                         "scenarios": scens, "convthresh": convthresh, "final_conv": r["conv"],
                         "Eobj": r["Eobj"], "trivial_bound": r["trivial_bound"]}}
    # N=1: the same run on one rank, bounded to n1_iters PH
    # iterations (about 10 s of CPU work at ~1.2k solves/s)
    try:
        t1 = time.perf_counter()
        r1 = ph_dist.run(1, scens, crops=c, rho=1.0, convthresh=convthresh, limit=n1_iters)
        out["n1"] = {"value": round(r1["subproblem_solves"] / r1["seconds_to_tol"], 2), "unit": "solves/s",
                     "cores": 1, "sample": f"the same oracle PH on 1 rank, {scens} scenarios, Iter0 + "
                                           f"{r1['iterations']} PH iterations ({r1['subproblem_solves']} "
                                           f"solves in {r1['seconds_to_tol']:.2f} s; "
                                           f"{time.perf_counter() - t1:.1f} s with start-up)"}
    except Exception as e:
        out["n1"] = {"value": None, "error": repr(e)}
    out["host"] = host_cpu_info()
    if f3_crops > 0:
        try:
            out["f3_subproblems"] = cpu_subproblem_rate(f3_crops, f3_sample, f3_seconds, cores)
        except Exception as e:  # the F3 sample must not kill the baseline
            out["f3_subproblems"] = {"value": None, "error": repr(e)}
    return out


def cgroup_cpu_quota():
    """CPUs this job may use by its cgroup (cpu.max quota / period), or None
    when unlimited or unreadable.  The GPU box's job cgroup allows 16 CPUs of
    its 2 x 64-core host (cpu.max "1600000 100000"), so more gloo ranks than
    that would only time-slice the same 16 CPUs."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q == "max":
            return None
        return max(1, int(int(q) // int(per)))
    except Exception:
        return None


def job_cpus():
    """The CPUs available to this job: the affinity mask capped by the
    cgroup quota (SURVEY 8(d)'s "all cores" of the host, as far as the job
    may use them)."""
    n = len(os.sched_getaffinity(0))
    q = cgroup_cpu_quota()
    return min(n, q) if q else n


def host_cpu_info():
    """lscpu of the host the CPU baseline ran on (record N and
    lscpu) and the CPUs this process may use."""
    import subprocess
    info = {"affinity_cpus": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(),
            "cgroup_cpu_quota": cgroup_cpu_quota()}
    try:
        txt = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        keep = ("Model name", "CPU(s)", "Thread(s) per core", "Core(s) per socket", "Socket(s)",
                "NUMA node(s)", "CPU max MHz", "L3 cache")
        for ln in txt.splitlines():
            k, _, v = ln.partition(":")
            if k.strip() in keep:
                info[k.strip()] = v.strip()
    except Exception as e:  # lscpu missing: say so
        info["lscpu_error"] = repr(e)
    return info


def vs_cpu(gpu_tol, cpu):
    """The like-for-like GPU / CPU comparison: PH from Iter0 to convthresh on
    the SAME farmer instance (cpu_baseline's sample size), wall seconds on
    the CPU baseline's ranks over the GPU's; and the subproblem solve rates of
    those two runs."""
    if not gpu_tol or not cpu or not cpu.get("ph_to_tol") or not gpu_tol.get("seconds"):
        return None
    c = cpu["ph_to_tol"]
    g_solves = gpu_tol["scenarios"] * (gpu_tol["ph_iterations"] + 1)
    return {"ph_to_tol_speedup": round(c["seconds"] / gpu_tol["seconds"], 1),
            "solves_per_s_ratio": round(g_solves / gpu_tol["seconds"] / cpu["value"], 1),
            "gpu_seconds": gpu_tol["seconds"], "cpu_seconds": c["seconds"], "cpu_cores": cpu["cores"],
            "scenarios": gpu_tol["scenarios"],
            "same_iterations": gpu_tol["ph_iterations"] == c["ph_iterations"],
            "basis": "PH wall-clock from Iter0 to convthresh on the same instance: the oracle PH (exact "
                     "HiGHS subproblem solves, no Pyomo overhead) on cpu_cores gloo ranks of the GPU "
                     "box's host against one MI355X"}


def workload_tag(kind, S_loc, c=None):
    """The workload tag tools/pmc_summary.py writes into a PMC summary
    (farmer10k_c1, farmer10k_c100, farmer1k_c1000, sslp10k), or None for a
    size no committed profile describes."""
    if S_loc % 1000 or S_loc == 0:
        return None
    return f"farmer{S_loc // 1000}k_c{c}" if kind == "farmer" else f"sslp{S_loc // 1000}k"


def pmc_traffic(kname, tag):
    """HBM bytes per launch of `kname` from the committed rocprofv3 PMC passes
    (profiles/r*/pmc_summary*.json, written by tools/pmc_summary.py from
    separate FETCH_SIZE / WRITE_SIZE passes of a bench command that ran only
    this workload, gfx950 FETCH_SIZE x2 correction applied there), matched on
    the summary's workload tag (the newest round first); else None."""
    import glob
    if tag is None:
        return None, None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_summary*.json")),
                       reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        k = d.get("kernels", {}).get(kname)
        if k and d.get("workload") == tag:
            return k.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    return None, None


def pmc_solve_traffic(kernels, tag):
    """HBM bytes per solve call of the listed kernels (bytes per launch x
    launches per solve, both from the newest committed PMC summary of the
    workload); None when the summary lacks one of them."""
    import glob
    if tag is None:
        return None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_summary*.json")),
                       reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("workload") != tag:
            continue
        ks = d.get("kernels", {})
        if not all(k in ks and ks[k].get("hbm_bytes_per_launch") is not None for k in kernels):
            return None
        return round(sum(ks[k]["hbm_bytes_per_launch"] * ks[k]["launches_per_solve"] for k in kernels))
    return None


def _progress(msg):
    """A progress line on stderr (long profiled runs must keep writing)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


class _heartbeat:
    """A progress line on stderr every `every` s while a long phase runs (a
    GPU call that writes nothing for 3 minutes is taken to be hung)."""

    def __init__(self, what, every=45.0):
        import threading
        self.what, self.every = what, every
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        t0 = time.perf_counter()
        while not self._stop.wait(self.every):
            print(f"[bench] {self.what}: {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    def __enter__(self):
        self._t.start()
        return self

    def __exit__(self, *a):
        self._stop.set()
        self._t.join()
        return False


def _red_dev():
    """Device of the timing max-reductions: the GPU under RCCL, host under gloo."""
    if dist.is_initialized() and dist.get_backend() == "gloo":
        return "cpu"
    return "cuda"


FP64_VECTOR_PEAK_TFS = 78.6  # MI355X FP64 vector, AMD spec (the microarch guide has no FP64 row)


def pdhg_flops_per_step(c):
    """Algorithmic FP64 flops of one PDHG step of one scenario: SpMV^T and
    SpMV (2 flops per entry each) + the column update (g - A'y, the prox
    step, the clip, the reflection and the Halpern average: 10 per column)
    + the row update (the dual prox, reflection, average: 10 per row)."""
    n, m, nnz = farmer_dims(c)
    return 4 * nnz + 10 * n + 10 * m


def hbm_config(args, world, farmer, PH, opts):
    """F3: farmer c=--hbm-crops, --scens scenarios per rank (the mid-size
    path: PDHG phase kernels mid_kernel and LDL' polish phases
    mid_polish_kernel).  Iter0, --warmup PH
    iterations (as the headline config), then --hbm-steps PH iterations
    through the device loop with the library's per-launch HIP events.

    roofline: the solve (all its phase launches) as the unit -- algorithmic
    bytes = every scenario's data in and solution out (the bytes the solve
    must move); `traffic` = the PMC-measured HBM bytes of the same phase
    launches per PH iteration.  `on_chip`: the PDHG phase kernel's FP64 rate
    (algorithmic flops per PDHG step x steps taken) against the FP64 vector
    peak.  `streaming_equivalent`: what a PDHG that streamed every step's
    operands from HBM would need (SURVEY 8(d) B_it) -- a work rate, not a
    bandwidth measurement."""
    c = args.hbm_crops
    S = args.scens * world
    names = [f"scen{i}" for i in range(S)]
    o = dict(opts)
    ph = PH(o, names, farmer.scenario_creator, scenario_creator_kwargs={"crops_multiplier": c})
    ph.PH_Prep()
    ph.subproblem_creation()
    ph._create_solvers()
    b = ph.batch
    torch.cuda.synchronize()
    _progress("F3 Iter0")
    t0 = time.perf_counter()
    ph.Iter0()
    torch.cuda.synchronize()
    t_iter0 = time.perf_counter() - t0
    nonopt0 = b.summary()[0]
    # the same warmup as the headline config (--warmup PH iterations)
    wu = max(1, args.warmup)
    ph.run_device_loop(0, wu, -1.0, chunk=1)
    ph.PHoptions["device_loop_graphs"] = False
    b.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph.run_device_loop(wu, wu + args.hbm_steps, -1.0, chunk=args.hbm_steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n_t, as_ms, po_ms, pd_ms, nk, k_ms, np_, p_ms = b.read_timing_full()
    st = b.loop_status()
    b.set_timing(False)
    d = torch.tensor([dt], dtype=torch.float64, device=_red_dev())
    if world > 1:
        dist.all_reduce(d, op=dist.ReduceOp.MAX)
    dt = float(d.item())
    nt = max(n_t, 1)
    n, m, nnz = farmer_dims(c)
    # one solve call: the transposes into the scenario-slowest layout, the
    # phase kernels, the transposes back and the bound pass (HIP events
    # around the whole mid_solve launch sequence)
    solve_ms = (as_ms + po_ms + pd_ms) / nt
    steps = st[4] / nt                                                # PDHG steps per solve call
    alg = ph.S_loc * solve_bytes_per_scenario(c)
    gbs = alg / (solve_ms / 1000.0) / 1e9
    stream_bytes = steps * bytes_per_pdhg_iter(c) + alg
    kern_ms = k_ms / max(nk, 1)
    tfs = (steps * pdhg_flops_per_step(c)) / (k_ms / nt / 1000.0) / 1e12 if k_ms > 0 else 0.0
    traffic = pmc_solve_traffic(("t_gather_kernel", "mid_kernel", "mid_polish_kernel", "t_scatter_kernel",
                                 "bound_kernel"), workload_tag("farmer", ph.S_loc, c))
    return {"workload": f"farmer PH, {S} scenarios ({args.scens} per GPU), crops_multiplier={c} "
                        f"(n={n}, m={m}, nnz={nnz} per scenario), rho={args.rho}",
            "value": round(S * args.hbm_steps / dt, 2), "unit": "solves/s",
            "ms_per_step": round(dt / args.hbm_steps * 1000.0, 3), "steps": args.hbm_steps,
            "iter0_s": round(t_iter0, 3), "iter0_not_optimal": nonopt0,
            "pdhg_steps_per_solve": round(st[4] / max(st[3], 1), 1), "pdhg_steps_max": st[5],
            "roofline": {"bound": "hbm", "kernel": "mid-size solve (t_gather_kernel transposes, mid_kernel "
                                                  "PDHG phases, mid_polish_kernel polish phases, "
                                                  "t_scatter_kernel, bound_kernel)",
                         "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "solve_ms": round(solve_ms, 3), "alg_bytes_per_solve": round(alg),
                         "launches_per_solve": {"mid_kernel": round(nk / nt, 2),
                                                "mid_polish_kernel": round(np_ / nt, 2)},
                         "kernel_ms": {"mid_kernel": round(kern_ms, 4),
                                       "mid_polish_kernel": round(p_ms / max(np_, 1), 4)},
                         "note": "algorithmic bytes = each scenario's data in + solution out "
                                 "(the scenario stays on chip between PDHG steps); traffic = "
                                 "rocprofv3 PMC bytes of the same kernels per solve call"},
            "on_chip": {"bound": "fp64-vector", "kernel": "mid_kernel",
                        "flops_per_step_per_scenario": pdhg_flops_per_step(c),
                        "achieved": round(tfs, 3), "peak": FP64_VECTOR_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": round(tfs / FP64_VECTOR_PEAK_TFS, 4)},
            "streaming_equivalent": {"bytes_per_solve": round(stream_bytes),
                                     "GBps": round(stream_bytes / (solve_ms / 1000.0) / 1e9, 1),
                                     "note": "SURVEY 8(d) B_it per scenario-step x steps taken: "
                                             "the bandwidth a PDHG streaming every step's operands "
                                             "from HBM would need -- a work rate, not a measurement"}}


def f4_bracket(ph, iters, trivial_bound, ef):
    """The bracket around the published EF after the bench's PH window (its
    W and x-bar): post_solve_bound (phbase.py:753-801: W on, prox off, the LP
    bound) <= EF <= the implementable x-bar objective (every scenario at the
    consensus first stage, W and prox off: the xhat of
    extensions/xhatbase.py).  Both are valid at any PH iteration; the EF
    (-1.334838651e8, paperruns/scripts/farmer/ef_1000_1000.out:183) must lie
    between them (`ok`)."""
    _progress("F4 EF bracket (x-bar objective, post_solve_bound)")
    t0 = time.perf_counter()
    ph._PHIter = iters
    ph.conv = float(ph.conv_hist[iters - 1].item()) if iters > 0 else None
    xb = ph.xbar.view(ph.K, ph.S_loc)[:, 0].cpu().numpy()
    ph._save_nonants()
    ph._fix_nonants(xb)
    kw = ph.solve_loop_launch(solver_options={"pdhg_max_iters": 100000}, dis_W=True, dis_prox=True)
    ph.solve_loop_finish(kw)
    xh_ok = bool((ph.batch.status == 0).all().item())
    wd, pd = ph.W_disabled, ph.prox_disabled
    ph._disable_W_and_prox()
    xhat = ph.Eobjective() if xh_ok else None
    ph.W_disabled, ph.prox_disabled = wd, pd
    ph._set_flags()
    ph._restore_nonants()
    with contextlib.redirect_stdout(sys.stderr):  # (its reference warning: stdout holds the one JSON line)
        psb = ph.post_solve_bound()
    torch.cuda.synchronize()
    out = {"after_ph_iterations": iters, "trivial_bound": trivial_bound, "post_solve_bound": psb,
           "xbar_objective": xhat, "published_ef": ef, "seconds": round(time.perf_counter() - t0, 2)}
    if ef is not None:
        out["ok"] = bool(psb <= ef + 1e-9 * abs(ef) and trivial_bound <= ef + 1e-9 * abs(ef)
                         and xhat is not None and ef <= xhat + 1e-9 * abs(ef))
        out["width_rel"] = None if xhat is None else (xhat - psb) / abs(ef)
    return out


def big_config(args, world, farmer, PH, opts):
    """farmer crops_multiplier --f4-crops (1000: n=12,000,
    m=9,001, nnz=27,000 per scenario), --f4-scens scenarios per rank (1000,
    the published EF's size), through the big path (csrc/solve_big.inc: the
    streaming PDHG with its state in HBM, the LDL' polish).  Iter0, one PH
    iteration of warmup, then --hbm-steps timed PH iterations (eager device
    loop) with the library's per-launch HIP events.

    roofline: the big_kernel (PDHG phase) as the dominant streaming kernel:
    algorithmic bytes = SURVEY 8(d) B_it = 8 (2 nnz + 7 n + 5 m) per
    scenario-step x the PDHG steps its launches took, over its launch time;
    `traffic` = the PMC-measured bytes of the same launches when a profile
    of this workload is committed.  The trivial bound is a lower bound of the
    published EF (-1.334838651e8 at S=1000, c=1000,
    paperruns/scripts/farmer/ef_1000_1000.out:183)."""
    c = args.f4_crops
    S = args.f4_scens * world
    o = dict(opts)
    ph = PH(o, [f"scen{i}" for i in range(S)], farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": c})
    ph.PH_Prep()
    ph.subproblem_creation()
    ph._create_solvers()
    b = ph.batch
    torch.cuda.synchronize()
    _progress("F4 Iter0")
    t0 = time.perf_counter()
    tb = ph.Iter0()
    torch.cuda.synchronize()
    t_iter0 = time.perf_counter() - t0
    nonopt0 = b.summary()[0]
    ph.PHoptions["device_loop_graphs"] = False
    ph.run_device_loop(0, 1, -1.0, chunk=1)
    b.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph.run_device_loop(1, 1 + args.hbm_steps, -1.0, chunk=args.hbm_steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n_t, _, _, _, nk, k_ms, np_, p_ms = b.read_timing_full()
    st = b.loop_status()
    b.set_timing(False)
    d = torch.tensor([dt], dtype=torch.float64, device=_red_dev())
    if world > 1:
        dist.all_reduce(d, op=dist.ReduceOp.MAX)
    dt = float(d.item())
    bracket = (f4_bracket(ph, 1 + args.hbm_steps, tb, -1.334838651e8 if (S == 1000 and c == 1000) else None)
               if args.f4_bracket else None)
    n, m, nnz = b.n, b.m, b.nnz
    bit = 8 * (2 * nnz + 7 * n + 5 * m)
    steps = st[4]
    gbs = steps * bit / (k_ms / 1000.0) / 1e9 if k_ms > 0 else 0.0
    # a PDHG phase is a big_kernel launch (one block per scenario) and a
    # big_team_kernel launch (a short list on teams); one of them exits at
    # once, and the phase events time both
    tag = workload_tag("farmer", ph.S_loc, c)
    t_one, t_team = pmc_traffic("big_kernel", tag)[0], pmc_traffic("big_team_kernel", tag)[0]
    trf = None if t_one is None and t_team is None else (t_one or 0) + (t_team or 0)
    return {"workload": f"farmer PH, {S} scenarios ({args.f4_scens} per GPU), crops_multiplier={c} "
                        f"(n={n}, m={m}, nnz={nnz} per scenario), rho={args.rho}",
            "value": round(S * args.hbm_steps / dt, 2), "unit": "solves/s",
            "ms_per_step": round(dt / args.hbm_steps * 1000.0, 3), "steps": args.hbm_steps,
            "iter0_s": round(t_iter0, 3), "iter0_not_optimal": nonopt0, "trivial_bound": tb,
            "published_ef": -1.334838651e8 if (S == 1000 and c == 1000) else None,
            "ef_bracket": bracket,
            "pdhg_steps_per_solve": round(steps / max(st[3], 1), 1), "pdhg_steps_max": st[5],
            "polished_per_solve": round(st[6] / max(st[3], 1), 3), "not_optimal_in_window": st[2],
            "roofline": {"bound": "hbm", "kernel": "big_kernel + big_team_kernel (a PDHG phase launch)",
                         "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4),
                         "traffic": None if trf is None or not nk else round(trf),
                         "alg_bytes_per_scenario_step": bit, "pdhg_steps": steps,
                         "kernel_ms": round(k_ms, 3), "launches": nk,
                         "polish_ms": round(p_ms, 3), "polish_launches": np_,
                         "note": "achieved = SURVEY 8(d) B_it x PDHG steps of the window / the "
                                 "PDHG phase launches' HIP-event time (big_kernel + big_team_kernel); "
                                 "traffic = their PMC bytes per phase"}}


def sslp_config(args, world, PH, opts):
    """BASELINE config 5: sslp_15_45 LP relaxation (n=705, m=60, nnz=1364 per
    scenario; synthetic scenarios, ClientPresent ~ Bernoulli(0.5) seeded per
    scenario, `mpisppy_amd/examples/sslp.py`), --sslp-scens per rank, rho 1.  Iter0, --warmup PH
    iterations, then --hbm-steps timed PH iterations through the device loop
    (eager: mid-size batch)."""
    from mpisppy_amd.examples import sslp as ex
    S = args.sslp_scens * world
    o = dict(opts)
    ph = PH(o, ex.scenario_names(S), ex.scenario_creator,
            scenario_creator_kwargs={"instance": "sslp_15_45_synthetic"})
    ph.PH_Prep()
    ph.subproblem_creation()
    ph._create_solvers()
    b = ph.batch
    torch.cuda.synchronize()
    _progress("sslp Iter0")
    t0 = time.perf_counter()
    ph.Iter0()
    torch.cuda.synchronize()
    t_iter0 = time.perf_counter() - t0
    nonopt0 = b.summary()[0]
    wu = max(1, args.warmup)
    ph.run_device_loop(0, wu, -1.0, chunk=1)
    ph.PHoptions["device_loop_graphs"] = False
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph.run_device_loop(wu, wu + args.hbm_steps, -1.0, chunk=args.hbm_steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = b.loop_status()
    d = torch.tensor([dt], dtype=torch.float64, device=_red_dev())
    if world > 1:
        dist.all_reduce(d, op=dist.ReduceOp.MAX)
    dt = float(d.item())
    return {"workload": f"sslp_15_45 LP relaxation PH, {S} synthetic scenarios ({args.sslp_scens} "
                        f"per GPU), n={b.n}, m={b.m}, nnz={b.nnz} per scenario, rho=1",
            "value": round(S * args.hbm_steps / dt, 2), "unit": "solves/s",
            "ms_per_step": round(dt / args.hbm_steps * 1000.0, 3), "steps": args.hbm_steps,
            "warmup": wu, "iter0_s": round(t_iter0, 3), "iter0_not_optimal": nonopt0,
            "not_optimal_in_window": st[2],
            "pdhg_steps_per_solve": round(st[4] / max(st[3], 1), 1), "pdhg_steps_max": st[5]}


def uc_config(args, world, PH, opts):
    """BASELINE config 4's model and cylinder structure at a reduced
    scenario count: the LP relaxation of paperruns/larger_uc/ReferenceModel_OK.py
    on the WECC-240 data (examples/uc.py: n = 56,869, m = 69,902,
    nnz = 240,508 per scenario; Scenario1.. of 1000scenarios_wind, the
    reference's rho setter), --uc-scens per rank, run as
    examples/uc/uc_cylinders.py runs it: a PH hub (:86) with a Lagrangian
    outer-bound spoke (:138-159) through spin_the_wheel (:167), the spoke
    asynchronous on a stream of its own (an xhat spoke's fixed-UnitOn LPs
    take past 400k PDHG steps each on this path: not in the line),
    1 + --uc-steps hub iterations.  The big path with y in the workspace
    slice, PDHG only (the LDL' factorisation, 58M update contributions, is
    past the big polish's size limit; DESIGN 4.11 records the interior-point
    attempt) on teams of blocks.  ms per PH iteration = the hub's solve_loop
    wall time per iteration (spokes overlapping); 1,000 scenarios are out of
    reach on this path (~400k PDHG steps per LP at ~10 MB per step)."""
    from mpisppy_amd.examples import uc
    from mpisppy_amd.phbase import PHBase
    from mpisppy_amd.cylinders.hub import PHHub
    from mpisppy_amd.cylinders.lagrangian_bounder import LagrangianOuterBound
    from mpisppy_amd.utils.sputils import spin_the_wheel
    S = args.uc_scens * world
    o = dict(opts)
    o["iter0_solver_options"] = {"pdhg_max_iters": 1000000}
    o["iterk_solver_options"] = {"pdhg_max_iters": 400000}
    o["xhat_max_iters"] = 400000
    o["device_loop"] = False
    iters = 1 + args.uc_steps
    base = dict(scenario_creator=uc.scenario_creator, all_scenario_names=uc.all_scenario_names(S),
                rho_setter=uc.scenario_rhos)
    hub_dict = {"hub_class": PHHub, "hub_kwargs": {"options": {"rel_gap": None}, "sync_every": 1,
                                                   "async_spokes": True},
                "opt_class": PH, "opt_kwargs": dict(PHoptions=dict(o, PHIterLimit=iters, convthresh=-1.0), **base)}
    spokes = [{"spoke_class": LagrangianOuterBound, "opt_class": PHBase,
               "opt_kwargs": dict(PHoptions=dict(o, PHIterLimit=iters), **base)}]
    _progress("UC hub + Lagrangian spoke")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(sys.stderr), _heartbeat("UC cylinders"):  # (stdout: the one JSON line)
        hub, _ = spin_the_wheel(hub_dict, spokes)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ph = hub.opt
    b = ph.batch
    log = list(ph.solve_log)   # (solves, seconds, ...) per solve_loop: Iter0 first
    t_iter0 = log[0][1] if log else float("nan")
    tk = [e[1] for e in log[1:1 + args.uc_steps]]
    d = torch.tensor([sum(tk)], dtype=torch.float64, device=_red_dev())
    if world > 1:
        dist.all_reduce(d, op=dist.ReduceOp.MAX)
    lag = hub.spokes[0]
    return {"workload": f"UC LP relaxation (ReferenceModel_OK.py, WECC-240), {S} scenarios "
                        f"({args.uc_scens} per GPU), n={b.n}, m={b.m}, nnz={b.nnz} per scenario, "
                        "reference rho setter; PH hub + Lagrangian spoke (uc_cylinders.py)",
            "iter0_s": round(t_iter0, 2), "trivial_bound": ph.trivial_bound,
            "ph_iterations": args.uc_steps,
            "ms_per_ph_iteration": round(float(d.item()) / max(len(tk), 1) * 1000.0, 1),
            "published_ms_per_ph_iteration": 910.0,
            "published_note": "examples/uc/quartz/10scen_nofw.baseline.out:8,107: iteration 1 at 29.25 s, "
                              "100 at 119.22 s -- the MIP, 10 scenarios on 30 ranks (2 nodes), gurobi",
            "lagrangian_bound": lag.bound, "best_outer_bound": hub.BestOuterBound,
            "not_optimal_after": int((b.status != 0).sum().item()),
            "wall_s": round(wall, 2),
            "parity": "unpinned (no reference file holds UC LP values); the oracle restatement matches "
                      "the Iter0 bounds to 2e-9 (tests/test_gpu_parity.py::test_uc_lp_relaxation_matches_oracle) "
                      "and the hub's outer bounds lie within 1 % below the oracle EF at 2 scenarios "
                      "(test_uc_hub_lagrangian_bracket_the_extensive_form)"}


def _spawn_ranks(n, cpu):
    """`bench.py --gpus N` without a launcher: this parent (which has not
    touched the GPU) starts N rank processes, one per GPU, with the
    torch.distributed env (127.0.0.1 rendezvous), hands rank 0 the CPU
    baseline it measured; returns the worst exit code and rank 0's JSON
    line."""
    import socket
    import subprocess
    import tempfile
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cpu_file = None
    if cpu is not None:
        fd, cpu_file = tempfile.mkstemp(prefix="bench_cpu_", suffix=".json")
        with os.fdopen(fd, "w") as f:
            json.dump(cpu, f)
    procs = []
    # (this process's fd 1 is stderr by now: rank 0's JSON comes back
    # through a pipe of its own)
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if cpu_file:
            env["BENCH_CPU_BASELINE_FILE"] = cpu_file
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=subprocess.PIPE if r == 0 else None))
    out0 = procs[0].communicate()[0]
    rcs = [procs[0].returncode] + [p.wait() for p in procs[1:]]
    if cpu_file:
        os.unlink(cpu_file)
    lines = [ln for ln in out0.decode().splitlines() if ln.startswith("{")]
    return max(abs(rc) for rc in rcs), (lines[-1] if lines else None)


def main():
    # fd 1 carries the JSON line only: everything else written to stdout, by
    # this process or by children that inherit it (the CPU baseline's gloo
    # ranks print from C++), goes to stderr
    json_fd = os.dup(1)
    os.dup2(2, 1)
    rc = _main()
    sys.stdout.flush()
    if isinstance(rc, str):
        os.write(json_fd, (rc + "\n").encode())
        rc = 0
    os.close(json_fd)
    sys.exit(rc or 0)


def _main():
    world = int(os.environ.get("WORLD_SIZE", "0"))
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    pre, _ = ap.parse_known_args()
    if world == 0 and pre.gpus > 1:
        # no launcher: measure the CPU baseline here (its workers fork before
        # any GPU use), then one process per GPU
        cpu = None if pre.no_cpu_baseline else _cpu_baseline_from_args()
        rc, line = _spawn_ranks(pre.gpus, cpu)
        return line if rc == 0 and line else rc
    out = run()
    return json.dumps(out) if out is not None else 0


def _parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scens", type=int, default=10000, help="scenarios per rank")
    ap.add_argument("--tol-scens", type=int, default=10000, help="scenarios of the PH-to-tol run")
    ap.add_argument("--crops", type=int, default=1)
    ap.add_argument("--rho", type=float, default=1.0)
    ap.add_argument("--tol-run", type=int, default=1, help="also time PH to convthresh")
    ap.add_argument("--convthresh", type=float, default=1e-4)
    ap.add_argument("--cpu-scens", type=int, default=200,
                    help="scenarios of the CPU-baseline oracle PH run (and of the GPU run beside it)")
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="CPU-baseline processes (the GPU box's CPU share is 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--hbm-crops", type=int, default=100,
                    help="crops_multiplier of the HBM-bound companion config (F3); 0 = skip")
    ap.add_argument("--hbm-steps", type=int, default=5)
    ap.add_argument("--graphs", type=int, default=0,
                    help="replay the timed device-loop chunk as a HIP graph (0: eager launches, "
                         "one ph_loop_pass call per PH iteration; -1: the library's 'auto', "
                         "graphs with the RCCL collective captured on several ranks -- not the "
                         "default: that capture has run on a one-rank RCCL group only)")
    ap.add_argument("--f4-scens", type=int, default=1000,
                    help="scenarios per rank of the F4 companion config (big path); 0 = skip")
    ap.add_argument("--f4-crops", type=int, default=1000)
    ap.add_argument("--f4-bracket", type=int, default=1,
                    help="F4: the EF bracket after the window (0: off, e.g. for a PMC window of the PH solves)")
    ap.add_argument("--sslp-scens", type=int, default=10000,
                    help="scenarios per rank of the sslp companion config (BASELINE config 5); 0 = skip")
    ap.add_argument("--uc-scens", type=int, default=2,
                    help="scenarios per rank of the UC companion config (BASELINE config 4's model); 0 = skip")
    ap.add_argument("--uc-steps", type=int, default=1, help="PH iterations of the UC companion")
    ap.add_argument("--only", choices=["f3", "f4", "sslp", "uc"], default=None,
                    help="profiling: run ONLY this companion config, exactly as the full line runs "
                         "it (its timed window is then the last --hbm-steps solve calls of the "
                         "process, the window tools/pmc_summary.py reads); prints its JSON")
    return ap


def _graphs_opt(args):
    return "auto" if args.graphs < 0 else bool(args.graphs)


def _cpu_baseline_from_args():
    args = _parser().parse_args()
    if args.no_cpu_baseline:
        return None
    try:
        return cpu_baseline(args.crops, args.cpu_scens, args.convthresh, args.cpu_cores,
                            args.hbm_crops)
    except Exception as e:  # the baseline must not kill the GPU number
        return {"value": None, "error": repr(e)}


def run():
    args = _parser().parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    cpu = None  # CPU baseline first: its worker processes fork before any GPU use
    if os.environ.get("BENCH_CPU_BASELINE_FILE"):
        if rank == 0:
            with open(os.environ["BENCH_CPU_BASELINE_FILE"]) as f:
                cpu = json.load(f)
    elif rank == 0 and world == 1:
        cpu = _cpu_baseline_from_args()
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
    if world > 1:
        # BENCH_DIST_BACKEND=gloo rehearses the multi-rank path with several
        # ranks on one GPU (RCCL refuses two ranks per device); default RCCL
        dist.init_process_group(os.environ.get("BENCH_DIST_BACKEND", "nccl")
                                if torch.cuda.is_available() else "gloo")
        if dist.get_world_size() != world:
            raise RuntimeError(f"process group has {dist.get_world_size()} ranks, WORLD_SIZE={world}")
        print(f"[bench] rank {rank}: {dist.get_world_size()} ranks over "
              f"{dist.get_backend()}", file=sys.stderr)

    import mpisppy_amd
    mpisppy_amd.disable_tictoc_output()
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer

    S, c = args.scens * world, args.crops  # weak scaling: --scens per rank
    if args.only:
        o1 = {"solvername": "mi355x_pdhg", "PHIterLimit": 100000, "defaultPHrho": args.rho,
              "convthresh": -1.0, "verbose": False, "display_progress": False,
              "display_timing": False, "iter0_solver_options": {}, "iterk_solver_options": {},
              "device_loop_graphs": False}
        res = {"f3": lambda: hbm_config(args, world, farmer, PH, o1),
               "f4": lambda: big_config(args, world, farmer, PH, o1),
               "sslp": lambda: sslp_config(args, world, PH, o1),
               "uc": lambda: uc_config(args, world, PH, o1)}[args.only]()
        if world > 1:
            dist.destroy_process_group()
        return {"only": args.only, args.only: res} if rank == 0 else None
    names = [f"scen{i}" for i in range(S)]
    opts = {"solvername": "mi355x_pdhg", "PHIterLimit": args.warmup + args.steps,
            "defaultPHrho": args.rho, "convthresh": -1.0, "verbose": False,
            "display_progress": False, "display_timing": False,
            "iter0_solver_options": {}, "iterk_solver_options": {},
            "device_loop_graphs": _graphs_opt(args)}
    _progress(f"building {S} scenarios (crops_multiplier {c})")
    ph = PH(opts, names, farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": c})
    ph.PH_Prep()
    ph.subproblem_creation()
    _progress("Iter0")
    ph.Iter0()
    _progress("warmup + timed PH iterations")

    # iterk_loop passes (phbase.py:1498-1553: Compute_Xbar -> Update_W ->
    # convergence_diff -> solve) queued on the device and replayed as one
    # HIP graph per `steps` iterations; convthresh off.  The warmup captures
    # the graph (same chunk) and runs `warmup` real iterations.
    ph.run_device_loop(0, args.warmup, -1.0, chunk=args.steps)
    b = ph.batch
    ph.solve_log.clear()
    # timed region: exactly `steps` PH iterations
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph.run_device_loop(args.warmup, args.warmup + args.steps, -1.0, chunk=args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt_local = time.perf_counter() - t0
    st1 = b.loop_status()
    dts = torch.tensor([dt_local], dtype=torch.float64, device=_red_dev())
    if world > 1:
        dist.all_reduce(dts, op=dist.ReduceOp.MAX)
    dt = float(dts.item())
    # (run_device_loop resets the device counters: st1 counts the timed steps)
    n_solves = st1[3]
    if n_solves != ph.S_loc * args.steps:
        raise RuntimeError(f"timed region solved {n_solves} scenarios, expected "
                           f"{ph.S_loc} x {args.steps}")
    tot_iters = float(st1[4])
    n_polished = float(st1[6])
    n_cached = float(st1[7])

    # kernel times: the next `steps` iterations of the same run, launched
    # eagerly with HIP events around the solve's kernels (library side, on
    # the stream they are launched on)
    ph.PHoptions["device_loop_graphs"] = False
    b.set_timing(True)
    ph.run_device_loop(args.warmup + args.steps, args.warmup + 2 * args.steps, -1.0,
                       chunk=args.steps)
    n_t, as_ms, po_ms, pd_ms, nk, k_ms, np_, p_ms = b.read_timing_full()
    fused = b.loop_fused()  # (the timing window's passes took the fused form)
    lk_n, lk_ms, lk_passes = b.loop_read_timing()
    sb_ = b.loop_status()
    b.set_timing(False)
    ph.PHoptions["device_loop_graphs"] = _graphs_opt(args)
    nt = max(n_t, 1)
    as_ms, po_ms, pd_ms = as_ms / nt, po_ms / nt, pd_ms / nt
    mid = (nk + np_) > 0      # a mid-size batch (--crops >= 6): its phase kernels instead
    t_iters = float(sb_[4]) / nt              # PDHG steps per solve call (all scenarios)
    t_pol = float(sb_[6]) / nt                # scenarios finished by a polish per call
    t_pdhg = float(sb_[3] - sb_[6] - sb_[7]) / nt  # scenarios left to PDHG per call

    S_loc = ph.S_loc
    K = 3 * c
    n, m, nnz = farmer_dims(c)
    cw = K + (K + 1) * 2 * (n + m)           # cache entry (doubles)
    sbw = 4 * n + 3 * m                      # static block (doubles)
    out_b = 8 * (n + m) + 4 + 4 + 16 + 40    # x, y, status, iters, pobj+dbound, diag
    # algorithmic bytes per launch (what the kernel must move at least):
    # active_set_kernel: every scenario's cache entry, static block,
    #   W/rho/xbar and flag in, the solution out
    as_bytes = S_loc * (8 * (cw + sbw + 3 * K) + 4 + out_b)
    # polish_kernel: per miss the static block, W/rho/xbar, hint, matrix
    #   values in; the solution and the refreshed cache entry out
    po_bytes = t_pol * (8 * (sbw + 3 * K + 4 + nnz + cw) + out_b)
    # tail_kernel (PDHG + rescue polish of the misses the register polish
    #   left): per scenario it solves the data in and the solution out +
    #   SURVEY 8(d) B_it per PDHG step
    pd_bytes = t_pdhg * solve_bytes_per_scenario(c) + t_iters * bytes_per_pdhg_iter(c)
    cand = [("active_set_kernel", as_ms, as_bytes), ("polish_kernel", po_ms, po_bytes),
            ("tail_kernel", pd_ms, pd_bytes)]
    if fused:
        # the fused pass (ph_loop_fused): the grouped cached-map kernel, then
        # finish_kernel = polish + tail + Compute_Xbar sums (per scenario K
        # x and probability reads) + the next pass's Update_W / convergence
        # (per slot: gid, W, rho, x in; xbar, xsqbar, W out; per scenario
        # absdiff out, its weight in)
        upd_bytes = S_loc * (K * (4 + 8 * 6) + 16) + S_loc * K * 16
        as_name = "active_set_g_kernel" if max(n, m) <= 32 else "active_set_kernel"
        cand = [(as_name, as_ms, as_bytes), ("finish_kernel", po_ms + pd_ms, po_bytes + pd_bytes + upd_bytes)]
    if mid:
        # per launch: a phase kernel's share of the solve's data in + solution
        # out is not separable, so each phase is priced at the whole solve's
        # algorithmic bytes (an upper bound of its rate)
        alg_solve = S_loc * solve_bytes_per_scenario(c)
        cand = [("mid_kernel", k_ms / max(nk, 1), alg_solve),
                ("mid_polish_kernel", p_ms / max(np_, 1), alg_solve)]
    persistent = lk_n > 0
    if persistent:
        # loop_kernel (ph_loop_run): the scenarios' cache entries, static
        # blocks, values and PH terms stay in LDS across the passes, so per
        # pass it must write, per scenario, x-bar / x-bar^2 / W (K each) and
        # absdiff, and the solution (x, y, status, iters, pobj, dbound, diag),
        # and per cache miss the refreshed entry + hint; per launch it loads
        # the resident data once.  Tails (PDHG) are the queued tail_kernel's.
        misses = (float(sb_[3] - sb_[7])) / max(lk_passes, 1)
        pass_bytes = S_loc * (8 * (3 * K + 1) + out_b) + misses * (8 * cw + 36)
        entry_bytes = S_loc * (8 * (cw + sbw + nnz + 6 * K + 1) + 8)
        lk_bytes = (pass_bytes * lk_passes + entry_bytes * lk_n) / lk_n
        cand = [("loop_kernel", lk_ms / lk_n, lk_bytes)]
    kname, kms, kbytes = max(cand, key=lambda t: t[1])
    achieved_gbs = kbytes / (kms / 1000.0) / 1e9 if kms > 0 else 0.0
    mean_iters = tot_iters / max(n_solves, 1)
    polished_frac = n_polished / max(n_solves, 1)
    cached_frac = n_cached / max(n_solves, 1)
    traffic, traffic_src = pmc_traffic(kname, workload_tag("farmer", S_loc, c))

    # PH wall-clock to convergence tolerance (fresh runs, same instance): the
    # 10k headline size, and the CPU baseline's sample size beside it
    def ph_to_tol(S_tol):
        opts2 = dict(opts)
        opts2["convthresh"] = args.convthresh
        opts2["PHIterLimit"] = 5000
        names2 = [f"scen{i}" for i in range(S_tol)]
        ph2 = PH(opts2, names2, farmer.scenario_creator,
                 scenario_creator_kwargs={"crops_multiplier": c})
        ph2.PH_Prep()
        ph2.subproblem_creation()
        ph2._create_solvers()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        tb = ph2.Iter0()
        ph2.iterk_loop()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t1
        w = torch.tensor([wall], dtype=torch.float64, device=_red_dev())
        if world > 1:
            dist.all_reduce(w, op=dist.ReduceOp.MAX)
        eobj = ph2.post_loops()
        return {"seconds": round(float(w.item()), 4), "ph_iterations": ph2._PHIter,
                "convthresh": args.convthresh, "final_conv": ph2.conv,
                "trivial_bound": tb, "Eobj": eobj, "scenarios": S_tol, "n_gpus": world}

    tol_info = tol_small = None
    _progress("timed region done")
    if args.tol_run:
        _progress("PH to tolerance")
        tol_info = ph_to_tol(args.tol_scens)
        if args.cpu_scens != args.tol_scens:
            tol_small = ph_to_tol(args.cpu_scens)

    # companion HBM-bound config: farmer crops_multiplier
    # 100, 10k scenarios per GPU -- the PDHG kernel's regime
    f3 = None
    if args.hbm_crops > 0:
        _progress("companion config F3")
        f3 = hbm_config(args, world, farmer, PH, opts)


    f4 = None
    if args.f4_scens > 0:
        _progress("companion config F4")
        f4 = big_config(args, world, farmer, PH, opts)

    sslp = None
    if args.sslp_scens > 0:
        _progress("companion config sslp")
        sslp = sslp_config(args, world, PH, opts)

    ucc = None
    if args.uc_scens > 0:
        _progress("companion config UC")
        ucc = uc_config(args, world, PH, opts)

    if rank == 0:
        value = S * args.steps / dt
        n, m, nnz = farmer_dims(c)
        out = {
            "metric": "scenario prox-QP solves/sec + PH wall-clock to conv tol (farmer 10k scens)",
            "value": round(value, 2),
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1000.0, 4),
            "higher_is_better": True,
            "scaling": "weak",
            # (BASELINE.md holds no published number for this metric)
            "vs_baseline": None,
            "vs_cpu": vs_cpu(tol_small, cpu),
            "dtype": "f64",
            "data": "synthetic (reference farmer generator, examples/farmer/farmer.py)",
            "config": {"workload": f"farmer PH, {S} scenarios ({args.scens} per GPU), crops_multiplier={c} "
                                   f"(n={n}, m={m}, nnz={nnz} per scenario), rho={args.rho}, "
                                   f"prox-QP to 1e-9 rel KKT, warm-started",
                       "scenarios": S, "scenarios_per_gpu": args.scens, "crops_multiplier": c,
                       "parallelism": f"scenario-sharded x{world} (one rank per GPU, RCCL allreduce)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel": kname,
                         "kernel_ms": round(kms, 4),
                         "alg_bytes_per_launch": round(kbytes),
                         "kernels": {k: {"ms": round(t, 4), "alg_bytes": round(bb),
                                         "GBps": round(bb / (t / 1000.0) / 1e9, 1) if t > 0 else None}
                                     for k, t, bb in cand},
                         "traffic_source": traffic_src,
                         "persistent": ({"launches": int(lk_n), "passes": int(lk_passes),
                                         "ms_per_pass_in_kernel": round(lk_ms / max(lk_passes, 1), 5)}
                                        if persistent else None),
                         "note": "per-launch averages from HIP events recorded by the library on "
                                 "the launch stream, over the `steps` PH iterations that follow "
                                 "the timed region (same run, eager launches); the dominant "
                                 "kernel by time is reported.  Algorithmic bytes: see DESIGN.md "
                                 "section 6 (loop_kernel, the persistent device loop: per pass the "
                                 "PH-term and solution writes of every scenario + the refreshed "
                                 "cache entries of the misses, per launch the resident data load; "
                                 "F2 is latency-bound and MALL-resident (SURVEY 8(d)); active_set: per scenario cache entry + static block "
                                 "+ W/rho/xbar in, solution out; polish: per cache miss; tail: per "
                                 "PDHG solve + SURVEY 8(d) B_it per PDHG step; mid-size batches: "
                                 "mid_kernel / mid_polish_kernel per launch, priced at the solve's "
                                 "data in + solution out)."},
            "pdhg_iters_per_solve": round(mean_iters, 2),
            "polished_fraction": round(polished_frac, 4),
            "cached_fraction": round(cached_frac, 4),
            "ph_to_tol": tol_info,
            "ph_to_tol_sample": tol_small,
            "cpu_baseline": cpu,
            "hbm_config": f3,
            "f4_config": f4,
            "sslp_config": sslp,
            "uc_config": ucc,
        }
    else:
        out = None
    if world > 1:
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
