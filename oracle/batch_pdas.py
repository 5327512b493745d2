"""Batched exact prox-QP solves + a single-process oracle PH for many small
scenarios (TEST INFRASTRUCTURE: generates golden PH trajectories; never
imported by the product).

The reference solves every scenario subproblem exactly with a commercial
solver (``mpisppy/phbase.py:946-988``).  ``oracle/solve.py`` restates that
with HiGHS + a KKT polish at ~3 ms per farmer subproblem, which makes a
10,000-scenario PH trajectory (millions of subproblems) a day of CPU time.
This module computes the same exact optima faster for scenarios that share
one small dense shape (farmer, ``examples/farmer/farmer.py:24-82``):

* every scenario keeps the active set of its last optimum (bounds / rows);
* the equality KKT system of that active set is solved for all scenarios at
  once (numpy batched LAPACK; the inverse is kept while the active set and
  the prox weights stay, so a PH iteration whose active sets hold costs two
  batched mat-vecs: solve + one refinement step);
* the clipped point must pass the same full KKT check as oracle/solve.py
  (``kkt_residual``, relative, default 1e-9; in practice ~1e-14);
* failures take primal-dual active-set rounds, and what still fails goes to
  ``oracle.solve.solve_scenario`` (HiGHS) one scenario at a time.

Which method found an optimum does not matter: the prox-QPs are strictly
convex in the nonants, and the KKT check certifies the point.  The PH driver
(`ph_run`) follows ``phbase.py:1364-1566`` exactly like ``oracle/ph_dist.py``
(Iter0 LPs, Compute_Xbar, Update_W, convergence_diff with the reference's
per-rank means for ``n_proc`` ranks, break before the solve, stale x at
Eobjective); tests pin the two against each other.

    python -m oracle.batch_pdas --scens 10000 --convthresh 1e-4 \
        --out tests/golden/farmer10k_ph.json
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np


def _kkt_err(x, y, g, q, A, rl, ru, l, u):
    """oracle/solve.py kkt_residual, one row per scenario: max(primal, dual)
    relative violation."""
    with np.errstate(invalid="ignore", over="ignore"):
        ax = np.einsum("sij,sj->si", A, x)
        scale_p = 1.0 + np.maximum(np.abs(x).max(1), np.abs(ax).max(1) if ax.size else 0.0)
        pv = np.zeros(x.shape[0])
        for v in (l - x, x - u):
            pv = np.maximum(pv, np.where(np.isfinite(v), v, -np.inf).max(1))
        if ax.size:
            for v in (rl - ax, ax - ru):
                pv = np.maximum(pv, np.where(np.isfinite(v), v, -np.inf).max(1))
        r = q * x + g - np.einsum("sij,si->sj", A, y)
        scale_d = 1.0 + np.abs(g).max(1)
        tol = (1e-9 * scale_p)[:, None]
        atl = np.isfinite(l) & (x - l <= tol * (1 + np.abs(l)))
        atu = np.isfinite(u) & (u - x <= tol * (1 + np.abs(u)))
        free = ~(atl | atu)
        dv = np.where(free, np.abs(r), 0.0).max(1)
        dv = np.maximum(dv, np.where(atl & ~atu, np.maximum(-r, 0.0), 0.0).max(1))
        dv = np.maximum(dv, np.where(atu & ~atl, np.maximum(r, 0.0), 0.0).max(1))
        if ax.size:
            rtl = np.isfinite(rl) & (ax - rl <= tol * (1 + np.abs(rl)))
            rtu = np.isfinite(ru) & (ru - ax <= tol * (1 + np.abs(ru)))
            dv = np.maximum(dv, np.where(~(rtl | rtu), np.abs(y), 0.0).max(1))
            dv = np.maximum(dv, np.where(rtl & ~rtu, np.maximum(-y, 0.0), 0.0).max(1))
            dv = np.maximum(dv, np.where(rtu & ~rtl, np.maximum(y, 0.0), 0.0).max(1))
    return np.maximum(pv / scale_p, dv / scale_d)


class BatchQP:
    """Exact solves of  min 1/2 x'diag(q_s)x + g_s'x  s.t. rl_s <= A_s x <= ru_s,
    l_s <= x <= u_s  for scenarios s of one shape (dense A_s)."""

    def __init__(self, scens, kkt_tol=1e-9, rounds=8, delta=1e-8, refine=30):
        self.scens = scens
        self.S = len(scens)
        self.m, self.n = scens[0].A.shape
        self.A = np.stack([sc.A.toarray() for sc in scens])
        self.l = np.stack([sc.l for sc in scens])
        self.u = np.stack([sc.u for sc in scens])
        self.rl = np.stack([sc.rl for sc in scens])
        self.ru = np.stack([sc.ru for sc in scens])
        self.eqc = np.isfinite(self.l) & (self.l == self.u)
        self.eqr = np.isfinite(self.rl) & (self.rl == self.ru)
        self.kkt_tol = kkt_tol
        self.rounds = rounds
        self.delta = delta
        self.refine = refine
        S, n, m = self.S, self.n, self.m
        self.atl = np.zeros((S, n), bool)
        self.atu = np.zeros((S, n), bool)
        self.rtl = np.zeros((S, m), bool)
        self.rtu = np.zeros((S, m), bool)
        self.M = None      # [S, N, N] KKT matrix of the kept active set
        self.Minv = None
        self.q_of_M = None
        self.stats = {"cached": 0, "factored": 0, "pdas_rounds": 0, "highs": 0}

    # ---------------------------------------------------------------
    def set_active_from(self, x, y, tau=1e-9):
        """Active set of a solution (bounds / rows within tau)."""
        l, u, rl, ru = self.l, self.u, self.rl, self.ru
        ax = np.einsum("sij,sj->si", self.A, x)
        with np.errstate(invalid="ignore"):
            self.atl = self.eqc | (np.isfinite(l) & (np.abs(x - l) <= tau * (1 + np.abs(l))))
            self.atu = ~self.atl & np.isfinite(u) & (np.abs(x - u) <= tau * (1 + np.abs(u)))
            self.rtl = self.eqr | (np.isfinite(rl) & (np.abs(ax - rl) <= tau * (1 + np.abs(rl))))
            self.rtu = ~self.rtl & np.isfinite(ru) & (np.abs(ax - ru) <= tau * (1 + np.abs(ru)))
        self.M = None

    def _system(self, idx, g, q):
        n, m = self.n, self.m
        A = self.A[idx]
        fixed = self.atl[idx] | self.atu[idx]
        act = self.rtl[idx] | self.rtu[idx]
        B = len(idx)
        M = np.zeros((B, n + m, n + m))
        M[:, :n, n:] = -np.transpose(A, (0, 2, 1)) * (~fixed)[:, :, None]
        M[:, n:, :n] = A * act[:, :, None]
        d = np.concatenate([np.where(fixed, 1.0, q[idx]), np.where(act, 0.0, 1.0)], axis=1)
        M[:, np.arange(n + m), np.arange(n + m)] += d
        # quasi-definite regularisation (oracle/solve.py _kkt_reg): +delta on
        # free columns, -delta on active rows; refinement against M removes it
        reg = np.concatenate([np.where(fixed, 0.0, self.delta), np.where(act, -self.delta, 0.0)], axis=1)
        return M, reg

    def _rhs(self, idx, g):
        l, u, rl, ru = self.l[idx], self.u[idx], self.rl[idx], self.ru[idx]
        atl, atu = self.atl[idx], self.atu[idx]
        rtl, rtu = self.rtl[idx], self.rtu[idx]
        xfix = np.where(atl, l, np.where(atu, u, 0.0))
        b = np.where(rtl, rl, np.where(rtu, ru, 0.0))
        return np.concatenate([np.where(atl | atu, xfix, -g[idx]), np.where(rtl | rtu, b, 0.0)],
                              axis=1)

    def _solve_idx(self, idx, g, q, use_cache):
        """Unclipped KKT solution (xu, y) of the kept active sets of idx;
        ok[idx] False where the system is singular."""
        n = self.n
        rhs = self._rhs(idx, g)
        if use_cache:
            M, Minv = self.M[idx], self.Minv[idx]
            self.stats["cached"] += len(idx)
        else:
            M, reg = self._system(idx, g, q)
            R = M.copy()
            N = M.shape[1]
            R[:, np.arange(N), np.arange(N)] += reg
            Minv = np.empty_like(M)
            ok = np.ones(len(idx), bool)
            try:
                Minv[:] = np.linalg.inv(R)
            except np.linalg.LinAlgError:
                for t in range(len(idx)):
                    try:
                        Minv[t] = np.linalg.inv(R[t])
                    except np.linalg.LinAlgError:
                        ok[t] = False
                        Minv[t] = 0.0
            ok &= np.all(np.isfinite(Minv), axis=(1, 2))
            self.stats["factored"] += len(idx)
            if self.M is None:
                N = M.shape[1]
                self.M = np.zeros((self.S, N, N))
                self.Minv = np.zeros((self.S, N, N))
                self.q_of_M = np.full((self.S, n), np.nan)
                self.cache_ok = np.zeros(self.S, bool)
            self.M[idx] = M
            self.Minv[idx] = Minv
            self.q_of_M[idx] = q[idx]
            self.cache_ok[idx] = ok
        z = np.einsum("sij,sj->si", Minv, rhs)
        scale = 1e-16 * (1.0 + np.abs(rhs).max(1))
        for _ in range(self.refine):  # iterative refinement against the exact system
            r = rhs - np.einsum("sij,sj->si", M, z)
            if np.all(np.abs(r).max(1) <= scale):
                break
            z += np.einsum("sij,sj->si", Minv, r)
        return z[:, :n], z[:, n:], self.cache_ok[idx].copy()

    def solve(self, g, q):
        """Exact optimum of every scenario: (x [S,n], y [S,m], err [S])."""
        S, n = self.S, self.n
        x = np.zeros((S, n))
        y = np.zeros((S, self.m))
        err = np.full(S, np.inf)
        todo = np.arange(S)
        fresh = self.M is None or not np.array_equal(self.q_of_M, q)
        for rnd in range(self.rounds):
            if todo.size == 0:
                break
            use_cache = (rnd == 0 and not fresh)
            if use_cache:
                hit = todo[self.cache_ok[todo]]
                miss = todo[~self.cache_ok[todo]]
                parts = [(hit, True), (miss, False)]
            else:
                parts = [(todo, False)]
            nxt = []
            for idx, uc in parts:
                if idx.size == 0:
                    continue
                xu, yu, ok = self._solve_idx(idx, g, q, uc)
                xc = np.minimum(np.maximum(xu, self.l[idx]), self.u[idx])
                e = _kkt_err(xc, yu, g[idx], q[idx], self.A[idx], self.rl[idx], self.ru[idx],
                             self.l[idx], self.u[idx])
                e = np.where(ok & np.all(np.isfinite(xc), 1) & np.all(np.isfinite(yu), 1), e, np.inf)
                acc = e <= self.kkt_tol
                x[idx[acc]] = xc[acc]
                y[idx[acc]] = yu[acc]
                err[idx[acc]] = e[acc]
                rej = idx[~acc]
                if rej.size:
                    # primal-dual active-set step from the unclipped point
                    # (oracle/solve.py _pdas rule)
                    xr, yr = xu[~acc], yu[~acc]
                    xr = np.where(np.isfinite(xr), xr, 0.0)
                    yr = np.where(np.isfinite(yr), yr, 0.0)
                    A = self.A[rej]
                    lam = q[rej] * xr + g[rej] - np.einsum("sij,si->sj", A, yr)
                    axu = np.einsum("sij,sj->si", A, xr)
                    l, u, rl, ru = self.l[rej], self.u[rej], self.rl[rej], self.ru[rej]
                    with np.errstate(invalid="ignore"):
                        self.atl[rej] = self.eqc[rej] | (np.isfinite(l) & (lam + (l - xr) > 0))
                        self.atu[rej] = ~self.atl[rej] & np.isfinite(u) & (-lam + (xr - u) > 0)
                        self.rtl[rej] = self.eqr[rej] | (np.isfinite(rl) & (yr + (rl - axu) > 0))
                        self.rtu[rej] = ~self.rtl[rej] & np.isfinite(ru) & (-yr + (axu - ru) > 0)
                    nxt.append(rej)
                    self.stats["pdas_rounds"] += rej.size
            todo = np.concatenate(nxt) if nxt else np.arange(0)
        if todo.size:
            from oracle.solve import solve_scenario
            for s in todo:
                sc = self.scens[s]
                xs, ys, feas = solve_scenario(g[s], q[s], sc.A, sc.rl, sc.ru, sc.l, sc.u,
                                              kkt_tol=self.kkt_tol)
                if not feas:
                    raise RuntimeError(f"scenario {sc.name} infeasible")
                x[s], y[s] = xs, ys
                err[s] = _kkt_err(xs[None], ys[None], g[s:s + 1], q[s:s + 1], self.A[s:s + 1],
                                  self.rl[s:s + 1], self.ru[s:s + 1], self.l[s:s + 1],
                                  self.u[s:s + 1])[0]
                self.stats["highs"] += 1
            # their active sets, for the next solve
            self._set_active_rows(todo, x[todo], y[todo])
            self.cache_ok[todo] = False
        return x, y, err

    def _set_active_rows(self, idx, x, y, tau=1e-9):
        l, u, rl, ru = self.l[idx], self.u[idx], self.rl[idx], self.ru[idx]
        ax = np.einsum("sij,sj->si", self.A[idx], x)
        with np.errstate(invalid="ignore"):
            atl = self.eqc[idx] | (np.isfinite(l) & (np.abs(x - l) <= tau * (1 + np.abs(l))))
            self.atl[idx] = atl
            self.atu[idx] = ~atl & np.isfinite(u) & (np.abs(x - u) <= tau * (1 + np.abs(u)))
            rtl = self.eqr[idx] | (np.isfinite(rl) & (np.abs(ax - rl) <= tau * (1 + np.abs(rl))))
            self.rtl[idx] = rtl
            self.rtu[idx] = ~rtl & np.isfinite(ru) & (np.abs(ax - ru) <= tau * (1 + np.abs(ru)))


def _slices(S, n):  # sputils.py:625-628
    avg = S / n
    return [range(int(i * avg), int((i + 1) * avg)) for i in range(n)]


def ph_run(scens, rho=1.0, convthresh=1e-4, limit=100000, n_proc=1, progress=False):
    """Oracle PH (phbase.py:1364-1566) over two-stage scenarios of one shape,
    probabilities 1/S (spbase.py:486-490).  convergence_diff is the
    reference's: per-rank mean |x - xbar| over the contiguous slices of
    `n_proc` ranks, summed, / n_proc (phbase.py:254-276)."""
    from oracle.solve import solve_scenario
    S = len(scens)
    K = len(scens[0].nonant_idx)
    idx = scens[0].nonant_idx
    p = 1.0 / S
    c = np.stack([sc.c for sc in scens])
    bq = BatchQP(scens)
    t0 = time.perf_counter()
    # Iter0 (phbase.py:1364-1470): LPs, exact vertices by HiGHS simplex
    x = np.zeros((S, bq.n))
    y = np.zeros((S, bq.m))
    for s, sc in enumerate(scens):
        xs, ys, feas = solve_scenario(sc.c, None, sc.A, sc.rl, sc.ru, sc.l, sc.u)
        if not feas:
            raise RuntimeError(f"scenario {sc.name} infeasible")
        x[s], y[s] = xs, ys
    tb = float(math.fsum(p * float(c[s] @ x[s]) for s in range(S)))
    bq.set_active_from(x, y)
    t_iter0 = time.perf_counter() - t0
    W = np.zeros((S, K))
    sl = _slices(S, n_proc)
    hist = []
    it = 0
    q = np.zeros((S, bq.n))
    q[:, idx] = rho
    xbar = np.zeros(K)
    for it in range(1, limit + 1):
        xn = x[:, idx]
        xbar = np.sum(p * xn, axis=0)                   # Compute_Xbar
        dx = xn - xbar
        W += rho * dx                                   # Update_W
        ad = np.abs(dx).sum(1)
        conv = sum(float(ad[r.start:r.stop].sum()) / (len(r) * K) for r in sl) / n_proc
        hist.append(conv)
        if progress and it % 200 == 0:
            print(f"[oracle PH] iter {it} conv {conv:.6e} {bq.stats}", file=sys.stderr)
        if conv < convthresh:
            break
        g = c.copy()
        g[:, idx] += W - rho * xbar
        x, y, err = bq.solve(g, q)
    t_tol = time.perf_counter() - t0
    xn = x[:, idx]
    eo = p * (np.einsum("sj,sj->s", c, x) + np.einsum("sk,sk->s", W, xn)
              + rho / 2.0 * np.sum(xn * xn - 2.0 * xbar * xn + xbar * xbar, axis=1))
    eobj = float(math.fsum(eo))
    return {"S": S, "rho": rho, "convthresh": convthresh, "n_proc": n_proc, "iterations": it,
            "conv": hist[-1], "conv_history": hist, "xbar": xbar.tolist(), "trivial_bound": tb,
            "Eobj": eobj, "W": W, "x_nonants": xn, "seconds_to_tol": t_tol,
            "seconds_iter0": t_iter0, "stats": dict(bq.stats)}


def golden(res, every=500):
    """The committed fixture: scalars, the xbar, every `every`-th scenario's
    W and nonants, every 100th conv value."""
    S = res["S"]
    pick = list(range(0, S, every))
    hist = res["conv_history"]
    return {"S": S, "rho": res["rho"], "convthresh": res["convthresh"], "n_proc": res["n_proc"],
            "iterations": res["iterations"], "conv": res["conv"],
            "conv_history_every100": {str(i + 1): hist[i] for i in range(99, len(hist), 100)},
            "conv_history_tail": hist[-5:], "xbar": res["xbar"],
            "trivial_bound": res["trivial_bound"], "Eobj": res["Eobj"],
            "W_abs_sum": float(np.abs(res["W"]).sum()),
            "W_sample": {str(s): res["W"][s].tolist() for s in pick},
            "x_nonants_sample": {str(s): res["x_nonants"][s].tolist() for s in pick}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scens", type=int, default=10000)
    ap.add_argument("--crops", type=int, default=1)
    ap.add_argument("--rho", type=float, default=1.0)
    ap.add_argument("--convthresh", type=float, default=1e-4)
    ap.add_argument("--n-proc", type=int, default=1)
    ap.add_argument("--limit", type=int, default=100000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import models as om
    scens = [om.farmer(f"scen{i}", a.crops) for i in range(a.scens)]
    t = time.time()
    res = ph_run(scens, a.rho, a.convthresh, a.limit, a.n_proc, progress=True)
    g = golden(res)
    g["crops_multiplier"] = a.crops
    g["generator"] = ("oracle/batch_pdas.py (batched exact active-set prox-QP solves, "
                      "KKT-checked; HiGHS fallback), " + " ".join(sys.argv[1:]))
    g["stats"] = res["stats"]
    g["wall_s"] = round(time.time() - t, 1)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(g, f, indent=1)
            f.write("\n")
    print(json.dumps({k: v for k, v in g.items()
                      if k not in ("W_sample", "x_nonants_sample", "conv_history_every100")}))


if __name__ == "__main__":
    main()
