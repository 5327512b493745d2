"""Oracle PH on N CPU ranks over torch.distributed gloo (TEST INFRASTRUCTURE
and the CPU baseline of bench.py).

The reference's `mpiexec -n N` run restated: every rank owns the contiguous
scenario slice ``sputils.py:625-628`` gives it and solves its scenarios one
after another (``phbase.py:1069-1079``) with the oracle's exact solver
(HiGHS 1.8 + KKT polish, oracle/solve.py); Compute_Xbar's node sums and
convergence_diff's per-rank means are allreduced (``phbase.py:198,274``);
Iter0 / iterk_loop follow ``phbase.py:1364-1566`` (break before the solve,
stale x at Eobjective).  Two-stage models (one ROOT node) only.

    python -m oracle.ph_dist --ranks 8 --scens 10000 --crops 1 --convthresh 1e-4 \
        --out tests/golden/farmer10k_ph.json
"""
import argparse
import json
import math
import os
import socket
import sys
import time

import numpy as np


def _slices(S, n):
    avg = S / n
    return [range(int(i * avg), int((i + 1) * avg)) for i in range(n)]


def _rank_main(rank, world, port, args, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = _ph(rank, world, args, dist, torch)
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


def _ph(rank, world, args, dist, torch):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle import models as om
    from oracle.solve import solve_scenario
    S = args.scens
    mine = list(_slices(S, world)[rank])
    scens = [om.farmer(f"scen{i}", args.crops) for i in mine]
    K = len(scens[0].nonant_idx)
    p = 1.0 / S  # spbase.py:486-490
    rho = args.rho
    x = [None] * len(scens)
    W = np.zeros((len(scens), K))
    xbar = np.zeros(K)

    def allreduce(v):
        t = torch.tensor(np.asarray(v, dtype=np.float64))
        dist.all_reduce(t)
        return t.numpy()

    def solve_all(w_on, prox_on):
        ob = 0.0
        for s, sc in enumerate(scens):
            g = sc.c.copy()
            qd = np.zeros_like(g)
            idx = sc.nonant_idx
            g[idx] += w_on * W[s] - prox_on * rho * xbar
            qd[idx] += prox_on * rho
            xs, _, feas = solve_scenario(g, qd, sc.A, sc.rl, sc.ru, sc.l, sc.u)
            if not feas:
                raise RuntimeError(f"scenario {sc.name} infeasible")
            x[s] = xs
            ob += p * (0.5 * float(qd @ (xs * xs)) + float(g @ xs)
                       + prox_on * rho / 2.0 * float(xbar @ xbar))
        return ob

    dist.barrier()
    t0 = time.perf_counter()
    tb = float(allreduce([solve_all(0.0, 0.0)])[0])       # Iter0, trivial bound
    t_iter0 = time.perf_counter() - t0
    hist = []
    it = 0
    for it in range(1, args.limit + 1):
        loc = np.zeros(2 * K)
        for s, sc in enumerate(scens):
            xn = x[s][sc.nonant_idx]
            loc[:K] += p * xn
            loc[K:] += p * xn * xn
        xbar = allreduce(loc)[:K]                           # Compute_Xbar
        d = 0.0
        for s, sc in enumerate(scens):                     # Update_W
            dx = x[s][sc.nonant_idx] - xbar
            W[s] += rho * dx
            d += float(np.sum(np.abs(dx)))
        conv = float(allreduce([d / (len(scens) * K)])[0]) / world   # convergence_diff
        hist.append(conv)
        if conv < args.convthresh:
            break
        solve_all(1.0, 1.0)
    t_tol = time.perf_counter() - t0
    # Eobjective at the (stale) x with W and prox on (phbase.py:279-312)
    eo = 0.0
    for s, sc in enumerate(scens):
        xs = x[s]
        xn = xs[sc.nonant_idx]
        eo += p * (float(sc.c @ xs) + float(W[s] @ xn)
                   + rho / 2.0 * float(np.sum(xn * xn - 2.0 * xbar * xn + xbar * xbar)))
    eobj = float(math.fsum(allreduce([eo])))
    # W of every 500th scenario (global index), gathered
    pick = [s for s, g in enumerate(mine) if g % 500 == 0]
    Wp = {int(mine[s]): W[s].tolist() for s in pick}
    allw = [None] * world
    dist.all_gather_object(allw, Wp)
    wabs = float(allreduce([float(np.sum(np.abs(W)))])[0])
    if rank != 0:
        return None
    Wsel = {}
    for dct in allw:
        Wsel.update({str(k): v for k, v in dct.items()})
    return {"S": S, "crops_multiplier": args.crops, "rho": rho, "convthresh": args.convthresh,
            "ranks": world, "iterations": it, "conv": hist[-1], "conv_history_tail": hist[-5:],
            "xbar": xbar.tolist(), "trivial_bound": tb, "Eobj": eobj, "W_sample": Wsel,
            "W_abs_sum": wabs, "seconds_to_tol": t_tol, "seconds_iter0": t_iter0,
            "subproblem_solves": S * (1 + max(it - 1, 0))}


def run(ranks, scens, crops=1, rho=1.0, convthresh=1e-4, limit=100000):
    """Oracle PH on `ranks` gloo processes; the rank-0 result dict."""
    import torch.multiprocessing as mp
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    args = argparse.Namespace(scens=scens, crops=crops, rho=rho, convthresh=convthresh, limit=limit)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, ranks, port, args, q)) for r in range(ranks)]
    for p in procs:
        p.start()
    import queue as _queue
    out = None
    while out is None:
        try:
            out = q.get(timeout=5)
        except _queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                for p in procs:
                    p.kill()
                raise RuntimeError("an oracle rank failed: "
                                   + str([p.exitcode for p in procs]))
    for p in procs:
        p.join()
        if p.exitcode != 0:
            raise RuntimeError(f"oracle rank exited with {p.exitcode}")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--scens", type=int, default=10000)
    ap.add_argument("--crops", type=int, default=1)
    ap.add_argument("--rho", type=float, default=1.0)
    ap.add_argument("--convthresh", type=float, default=1e-4)
    ap.add_argument("--limit", type=int, default=100000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    t = time.time()
    res = run(a.ranks, a.scens, a.crops, a.rho, a.convthresh, a.limit)
    res["wall_s"] = time.time() - t
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    print(json.dumps({k: v for k, v in res.items() if k not in ("W_sample",)}))


if __name__ == "__main__":
    main()
