"""CPU prototype (development tool, not product, not oracle) of the mid-size
active-set polish: a quasi-definite LDL' of the active set's KKT system with
a fill-reducing order fixed per sparsity pattern (computed once on the host,
shared by every scenario), static pivots, regularisation and iterative
refinement, inside primal-dual active-set (PDAS) rounds.

    python tools/kkt_ldl_proto.py [c] [scen]

Checks on farmer (crops_multiplier c): the symbolic sizes (nnz(L), etree
levels) and that the polish reproduces the HiGHS vertex / the exact prox-QP
from a perturbed active set.
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import models as om  # noqa: E402
from oracle.solve import solve_scenario, kkt_residual  # noqa: E402


def kkt_pattern(A):
    """Pattern of the (n+m) x (n+m) KKT matrix: diagonal + A and A'."""
    A = sp.csr_matrix(A)
    m, n = A.shape
    N = n + m
    adj = [set() for _ in range(N)]
    for i in range(m):
        for p in range(A.indptr[i], A.indptr[i + 1]):
            j = A.indices[p]
            adj[j].add(n + i)
            adj[n + i].add(j)
    return adj


def min_degree(adj):
    """Plain minimum-degree order (explicit elimination graph, ties by index)."""
    N = len(adj)
    g = [set(a) for a in adj]
    alive = np.ones(N, dtype=bool)
    order = []
    import heapq
    h = [(len(g[v]), v) for v in range(N)]
    heapq.heapify(h)
    while h:
        d, v = heapq.heappop(h)
        if not alive[v] or d != len(g[v]):
            continue
        alive[v] = False
        order.append(v)
        nb = list(g[v])
        for a in nb:
            g[a].discard(v)
        for a in nb:
            before = len(g[a])
            g[a].update(b for b in nb if b != a)
            if len(g[a]) != before or True:
                heapq.heappush(h, (len(g[a]), a))
        g[v] = set()
    return np.array(order)


def symbolic(adj, order):
    """L pattern (permuted indices), etree parent, levels."""
    N = len(adj)
    pos = np.empty(N, dtype=np.int64)
    pos[order] = np.arange(N)
    cols = [set() for _ in range(N)]
    for v in range(N):
        for a in adj[v]:
            i, j = pos[a], pos[v]
            if i > j:
                cols[j].add(i)
    parent = np.full(N, -1)
    for j in range(N):
        if cols[j]:
            p = min(cols[j])
            parent[j] = p
            cols[p].update(i for i in cols[j] if i > p)
    Lp = [sorted(c) for c in cols]
    level = np.zeros(N, dtype=np.int64)
    for j in range(N):
        if parent[j] >= 0:
            level[parent[j]] = max(level[parent[j]], level[j] + 1)
    return Lp, parent, level, pos


def ldl_numeric(Kp, Lp):
    """Left-looking LDL' without pivoting on the permuted matrix Kp (dict of
    columns {i: v} for i >= j).  Returns L (list of dict) and D."""
    N = len(Lp)
    L = [dict() for _ in range(N)]
    D = np.zeros(N)
    rows_of = [[] for _ in range(N)]  # k columns with L[i][k] != 0 for row i
    for j in range(N):
        col = dict(Kp[j])
        for k in rows_of[j]:
            ljk = L[k][j]
            f = ljk * D[k]
            for i, lik in L[k].items():
                if i >= j:
                    col[i] = col.get(i, 0.0) - lik * f
        d = col.get(j, 0.0)
        D[j] = d
        for i in Lp[j]:
            v = col.get(i, 0.0) / d
            L[j][i] = v
            rows_of[i].append(j)
    return L, D


def ldl_solve(L, D, b):
    N = len(D)
    z = b.copy()
    for j in range(N):
        zj = z[j]
        for i, v in L[j].items():
            z[i] -= v * zj
    z /= D
    for j in range(N - 1, -1, -1):
        s = z[j]
        for i, v in L[j].items():
            s -= v * z[i]
        z[j] = s
    return z


def polish(A, g, q, l, u, rl, ru, cs, rs, Lp, pos, delta=1e-9, refine=30):
    """Solve the KKT system of the active set (cs: 0 free / 1 at l / 2 at u;
    rs: 0 inactive / 1 at rl / 2 at ru) by regularised LDL' + refinement.
    Returns x, y (y > 0 <-> row at rl)."""
    A = sp.csr_matrix(A)
    m, n = A.shape
    N = n + m
    fixed = cs != 0
    xfix = np.where(cs == 1, l, np.where(cs == 2, u, 0.0))
    act = rs != 0
    b = np.where(rs == 1, rl, np.where(rs == 2, ru, 0.0))
    # true system T z = r  (symmetric):
    #   free j:  q_j x_j - sum_i A_ij y_i = -g_j
    #   fixed j: x_j = xfix_j
    #   active i: -sum_j A_ij x_j = -b_i  (+ fixed columns moved right)
    #   inactive i: -y_i = 0
    rhs = np.zeros(N)
    rhs[:n] = np.where(fixed, xfix, -g)
    Af = A.multiply(1.0).tocsr()
    bf = b - A @ np.where(fixed, xfix, 0.0)
    rhs[n:] = np.where(act, -bf, 0.0)
    rows, colsA, vals = [], [], []
    Acoo = A.tocoo()
    keep = (~fixed[Acoo.col]) & act[Acoo.row]
    ri, cj, av = Acoo.row[keep], Acoo.col[keep], Acoo.data[keep]
    Hd = np.where(fixed, 1.0, q)
    Gd = np.where(act, 0.0, -1.0)
    T = sp.coo_matrix((np.concatenate([Hd, Gd, -av, -av]),
                       (np.concatenate([np.arange(n), n + np.arange(m), cj, n + ri]),
                        np.concatenate([np.arange(n), n + np.arange(m), n + ri, cj]))),
                      shape=(N, N)).tocsr()
    Hr = Hd + np.where(fixed, 0.0, delta)
    Gr = Gd - np.where(act, delta, 0.0)
    Treg = T + sp.diags(np.concatenate([Hr - Hd, Gr - Gd]))
    # permuted lower columns
    P = sp.csr_matrix((np.ones(N), (pos, np.arange(N))), shape=(N, N))
    Tp = (P @ Treg @ P.T).tocsc()
    Kp = []
    for j in range(N):
        c = {}
        for p in range(Tp.indptr[j], Tp.indptr[j + 1]):
            i = Tp.indices[p]
            if i >= j:
                c[i] = Tp.data[p]
        Kp.append(c)
    L, D = ldl_numeric(Kp, Lp)
    if np.any(D == 0) or not np.all(np.isfinite(D)):
        bad = np.nonzero((D == 0) | ~np.isfinite(D))[0]
        print("zero/nonfinite pivots at", bad[:10], "orig", np.argsort(pos)[bad[:10]], "Kp diag",
              [Kp[j].get(j) for j in bad[:10]])
    z = np.zeros(N)
    hist = []
    for _ in range(refine):
        r = rhs - T @ z
        hist.append(np.abs(r).max() / (1 + np.abs(rhs).max()))
        if hist[-1] < 1e-16:
            break
        dz = ldl_solve(L, D, P @ r)
        z = z + P.T @ dz
    if os.environ.get("REFHIST"):
        print("     refinement", " ".join(f"{h:.1e}" for h in hist))
    x = z[:n]
    y = z[n:]
    return x, y, np.linalg.norm(rhs - T @ z) / (1 + np.linalg.norm(rhs))


def main():
    c = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    sn = int(sys.argv[2]) if len(sys.argv) > 2 else 109
    sc = om.farmer(f"scen{sn}", c)
    A = sc.A
    m, n = A.shape
    t = time.time()
    adj = kkt_pattern(A)
    order = min_degree(adj)
    Lp, parent, level, pos = symbolic(adj, order)
    nnzL = sum(len(x) for x in Lp)
    print(f"c={c}: n={n} m={m} nnz={A.nnz} N={n + m} nnz(L)={nnzL} levels={level.max() + 1} "
          f"symbolic {time.time() - t:.2f}s; per-level widths "
          f"{np.bincount(level)[:8]} ... {np.bincount(level)[-4:]}")
    # Iter0 LP exactly (HiGHS) -> its active set -> polish
    g = sc.c.copy()
    q = np.zeros(n)
    x0, y0, feas = solve_scenario(g, q, A, sc.rl, sc.ru, sc.l, sc.u)
    ax = A @ x0
    tol = 1e-9
    cs = np.where(np.isfinite(sc.l) & (np.abs(x0 - sc.l) <= tol * (1 + np.abs(sc.l))), 1,
                  np.where(np.isfinite(sc.u) & (np.abs(x0 - sc.u) <= tol * (1 + np.abs(sc.u))), 2, 0))
    rs = np.where(np.isfinite(sc.rl) & (np.abs(ax - sc.rl) <= tol * (1 + np.abs(sc.rl))) & (y0 > 0), 1,
                  np.where(np.isfinite(sc.ru) & (np.abs(ax - sc.ru) <= tol * (1 + np.abs(sc.ru))) & (y0 < 0), 2, 0))
    rs = np.where(sc.rl == sc.ru, 1, rs)
    print(f"active set: free cols {np.sum(cs == 0)}, active rows {np.sum(rs != 0)}")
    for delta in (1e-2, 1e-4, 1e-6):
        t = time.time()
        x, y, res = polish(A, g, q, sc.l, sc.u, sc.rl, sc.ru, cs, rs, Lp, pos, delta=delta)
        x = np.clip(x, sc.l, sc.u)
        pv, dv = kkt_residual(x, y, g, q, A, sc.rl, sc.ru, sc.l, sc.u)
        print(f"  LP delta {delta:.0e}: system residual {res:.2e}  KKT primal {pv:.2e} dual {dv:.2e} "
              f"obj {g @ x:.9f} vs {g @ x0:.9f}  |x-x0| {np.abs(x - x0).max():.2e} ({time.time() - t:.1f}s)")


if __name__ == "__main__":
    main()
