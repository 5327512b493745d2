"""Exact per-scenario LP / diagonal-QP solves for the oracle (TEST INFRASTRUCTURE).

The reference hands every scenario subproblem to a commercial solver via
Pyomo (``mpisppy/phbase.py:946-988``): simplex/barrier, i.e. an *exact*
optimum.  The oracle reproduces that with HiGHS 1.8.0 (the copy bundled in
scipy 1.15.3):

* LPs (Iter0, Lagrangian and post-solve bounds) -> HiGHS dual simplex with
  tightened tolerances: a vertex optimum, like CPLEX/Gurobi return.
* PH prox-QPs (``phbase.py:1133-1209``: min 1/2 x'diag(q)x + g'x) -> HiGHS
  QP, whose answer is only ~1e-6 accurate, is *polished*: the active set is
  read off the HiGHS point, the equality-constrained KKT system is solved in
  float64 and the result is accepted only if it passes a full KKT check.
"""
import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla
from scipy.optimize._highspy import _core as hc


class OracleSolveError(RuntimeError):
    pass


def _highs_solve(c, q, A, rl, ru, l, u, time_limit=20.0):
    A = sp.csc_matrix(A)
    m, n = A.shape
    lp = hc.HighsLp()
    lp.num_col_ = n
    lp.num_row_ = m
    lp.col_cost_ = np.asarray(c, dtype=np.float64)
    lp.col_lower_ = np.asarray(l, dtype=np.float64)
    lp.col_upper_ = np.asarray(u, dtype=np.float64)
    lp.row_lower_ = np.asarray(rl, dtype=np.float64)
    lp.row_upper_ = np.asarray(ru, dtype=np.float64)
    mat = hc.HighsSparseMatrix()
    mat.format_ = hc.MatrixFormat.kColwise
    mat.num_col_ = n
    mat.num_row_ = m
    mat.start_ = A.indptr.astype(np.int32)
    mat.index_ = A.indices.astype(np.int32)
    mat.value_ = A.data.astype(np.float64)
    lp.a_matrix_ = mat
    h = hc._Highs()
    h.setOptionValue("output_flag", False)
    h.setOptionValue("primal_feasibility_tolerance", 1e-10)
    h.setOptionValue("dual_feasibility_tolerance", 1e-10)
    h.setOptionValue("random_seed", 0)
    h.setOptionValue("time_limit", time_limit)  # a stuck solve fails loudly instead of hanging
    h.passModel(lp)
    if q is not None and np.any(q != 0):
        hs = hc.HighsHessian()
        hs.dim_ = n
        hs.format_ = hc.HessianFormat.kTriangular
        nz = np.nonzero(q)[0]
        start = np.zeros(n + 1, dtype=np.int32)
        cnt = np.zeros(n, dtype=np.int32)
        cnt[nz] = 1
        start[1:] = np.cumsum(cnt)
        hs.start_ = start
        hs.index_ = nz.astype(np.int32)
        hs.value_ = np.asarray(q, dtype=np.float64)[nz]
        h.passHessian(hs)
    else:
        h.setOptionValue("solver", "simplex")
    h.run()
    status = h.getModelStatus()
    sol = h.getSolution()
    global _last_basis
    try:
        bas = h.getBasis()
        _last_basis = (np.array([str(v).rsplit(".", 1)[-1] for v in bas.col_status]),
                       np.array([str(v).rsplit(".", 1)[-1] for v in bas.row_status])) \
            if bas.valid else None
    except Exception:  # pragma: no cover - basis not offered
        _last_basis = None
    return status, np.array(sol.col_value), np.array(sol.row_dual), np.array(sol.col_dual)


_last_basis = None


def _kkt_reg(c, q, A, rl, ru, l, u, atl, atu, rtl, rtu, delta=1e-8, refine=30):
    """Equality KKT system of an active set by a regularised sparse LU
    (quasi-definite: diag(q)+delta on free columns, -delta on active rows)
    plus iterative refinement against the unregularised system."""
    A = sp.csr_matrix(A)
    m, n = A.shape
    fixed = atl | atu
    xfix = np.where(atl, l, np.where(atu, u, 0.0))
    act = rtl | rtu
    b = np.where(rtl, rl, np.where(rtu, ru, 0.0))
    Ac = A.tocoo()
    keep = (~fixed[Ac.col]) & act[Ac.row]
    ri, cj, av = Ac.row[keep], Ac.col[keep], Ac.data[keep]
    Hd = np.where(fixed, 1.0, q)
    Gd = np.where(act, 0.0, -1.0)
    N = n + m
    T = sp.coo_matrix((np.concatenate([Hd, Gd, -av, -av]),
                       (np.concatenate([np.arange(n), n + np.arange(m), cj, n + ri]),
                        np.concatenate([np.arange(n), n + np.arange(m), n + ri, cj]))),
                      shape=(N, N)).tocsc()
    R = T + sp.diags(np.concatenate([np.where(fixed, 0.0, delta), np.where(act, -delta, 0.0)]))
    lu = spla.splu(R.tocsc())
    rhs = np.concatenate([np.where(fixed, xfix, -c),
                          np.where(act, -(b - A @ np.where(fixed, xfix, 0.0)), 0.0)])
    z = np.zeros(N)
    for _ in range(refine):
        r = rhs - T @ z
        if not np.all(np.isfinite(r)) or np.abs(r).max() <= 1e-16 * (1 + np.abs(rhs).max()):
            break
        z += lu.solve(r)
    return z[:n], z[n:]


def _basis_polish(c, q, A, rl, ru, l, u, kkt_tol, rounds=10):
    """Active set from HiGHS's final basis statuses (at lower / upper /
    basic), the KKT system solved exactly (_kkt_reg), then primal-dual
    active-set rounds.  Returns (err, x, y) of the best point or None."""
    if _last_basis is None:
        return None
    cs, rs = _last_basis
    if cs.size != c.size:
        return None
    eq = np.isfinite(l) & (l == u)
    atl = eq | (cs == "kLower")
    atu = ~atl & (cs == "kUpper")
    req = np.isfinite(rl) & (rl == ru)
    rtl = req | (rs == "kLower")
    rtu = ~rtl & (rs == "kUpper")
    A = sp.csr_matrix(A)
    best = None
    for _ in range(rounds):
        try:
            xu, yu = _kkt_reg(c, q, A, rl, ru, l, u, atl, atu, rtl, rtu)
        except RuntimeError:  # singular factor
            return best
        x = np.minimum(np.maximum(xu, l), u)
        if not np.all(np.isfinite(x)) or not np.all(np.isfinite(yu)):
            return best
        pv, dv = kkt_residual(x, yu, c, q, A, rl, ru, l, u)
        err = max(pv, dv)
        if best is None or err < best[0]:
            best = (err, x, yu)
        if err <= kkt_tol:
            return best
        lam = q * xu + c - A.T @ yu
        axu = A @ xu
        natl = eq | (np.isfinite(l) & (lam + (l - xu) > 0))
        natu = ~natl & np.isfinite(u) & (-lam + (xu - u) > 0)
        nrtl = req | (np.isfinite(rl) & (yu + (rl - axu) > 0))
        nrtu = ~nrtl & np.isfinite(ru) & (-yu + (axu - ru) > 0)
        if (np.array_equal(natl, atl) and np.array_equal(natu, atu)
                and np.array_equal(nrtl, rtl) and np.array_equal(nrtu, rtu)):
            return best
        atl, atu, rtl, rtu = natl, natu, nrtl, nrtu
    return best


def _qp_by_cuts(c, q, A, rl, ru, l, u, iters=400):
    """Approximate prox-QP point by Kelley cutting planes: each quadratic
    term 1/2 q_j x_j^2 becomes an epigraph column t_j >= q_j a x_j - q_j a^2/2
    over a growing set of tangent points a, solved as LPs by HiGHS simplex.
    Used only to seed the active set when HiGHS's own QP solver stalls (its
    time limit; seen on sslp_15_45_15 prox-QPs); the exact point then comes
    from the PDAS polish and the KKT check."""
    A = sp.csr_matrix(A)
    m, n = A.shape
    J = np.nonzero(q)[0]
    k = J.size
    pts = []
    for j in J:
        lo = l[j] if np.isfinite(l[j]) else -1e4
        hi = u[j] if np.isfinite(u[j]) else 1e4
        pts.append(list(np.linspace(lo, hi, 33)))
    x = None
    global _last_basis
    for _ in range(iters):
        rows, cols, vals, lo_, hi_ = [], [], [], [], []
        r = 0
        for t, j in enumerate(J):
            for a in pts[t]:
                # q a x_j - t_j <= q a^2 / 2
                rows += [r, r]
                cols += [j, n + t]
                vals += [q[j] * a, -1.0]
                lo_.append(-np.inf)
                hi_.append(0.5 * q[j] * a * a)
                r += 1
        C = sp.coo_matrix((vals, (rows, cols)), shape=(r, n + k)).tocsr()
        Ax = sp.vstack([sp.hstack([A, sp.csr_matrix((m, k))]), C]).tocsr()
        st, z, _, _ = _highs_solve(np.concatenate([c, np.ones(k)]), None, Ax,
                                   np.concatenate([rl, lo_]), np.concatenate([ru, hi_]),
                                   np.concatenate([l, np.full(k, -np.inf)]),
                                   np.concatenate([u, np.full(k, np.inf)]))
        if "Optimal" not in str(st):
            return x
        x, tt = z[:n], z[n:]
        gap = 0.5 * q[J] * x[J] ** 2 - tt
        if np.max(gap) <= 1e-14 * (1.0 + np.max(np.abs(c))):
            if _last_basis is not None:  # the original columns' and rows' statuses
                _last_basis = (_last_basis[0][:n], _last_basis[1][:m])
            break
        for t, j in enumerate(J):
            if gap[t] > 0:
                pts[t].append(x[j])
    return x


def kkt_residual(x, y, c, q, A, rl, ru, l, u):
    """Max relative KKT violation of (x, y) for min 1/2x'Qx+c'x (y>=0 <-> row at rl)."""
    A = sp.csr_matrix(A)
    ax = A @ x
    scale_p = 1.0 + np.max(np.abs(np.concatenate([x, ax])))
    pv = 0.0
    pv = max(pv, np.max(np.maximum(l - x, 0.0)), np.max(np.maximum(x - u, 0.0)))
    pv = max(pv, np.max(np.maximum(rl - ax, 0.0), initial=0.0),
             np.max(np.maximum(ax - ru, 0.0), initial=0.0))
    r = q * x + c - A.T @ y
    scale_d = 1.0 + np.max(np.abs(c))
    dv = 0.0
    tol = 1e-9 * scale_p
    atl = np.isfinite(l) & (x - l <= tol * (1 + np.abs(l)))
    atu = np.isfinite(u) & (u - x <= tol * (1 + np.abs(u)))
    free = ~(atl | atu)
    dv = max(dv, np.max(np.abs(r[free]), initial=0.0))
    dv = max(dv, np.max(np.maximum(-r[atl & ~atu], 0.0), initial=0.0))
    dv = max(dv, np.max(np.maximum(r[atu & ~atl], 0.0), initial=0.0))
    # complementarity of row duals
    rtl = np.isfinite(rl) & (ax - rl <= tol * (1 + np.abs(rl)))
    rtu = np.isfinite(ru) & (ru - ax <= tol * (1 + np.abs(ru)))
    dv = max(dv, np.max(np.abs(y[~(rtl | rtu)]), initial=0.0))
    dv = max(dv, np.max(np.maximum(-y[rtl & ~rtu], 0.0), initial=0.0))
    dv = max(dv, np.max(np.maximum(y[rtu & ~rtl], 0.0), initial=0.0))
    return pv / scale_p, dv / scale_d


def _polish(x0, c, q, A, rl, ru, l, u, tau):
    A = sp.csr_matrix(A)
    n = x0.size
    ax = A @ x0
    atl = np.isfinite(l) & (np.abs(x0 - l) <= tau * (1 + np.abs(l)))
    atu = np.isfinite(u) & (np.abs(x0 - u) <= tau * (1 + np.abs(u)))
    xb = np.where(atl, l, np.where(atu, u, 0.0))
    bnd = atl | atu
    F = np.nonzero(~bnd)[0]
    rtl = np.isfinite(rl) & (np.abs(ax - rl) <= tau * (1 + np.abs(rl)))
    rtu = np.isfinite(ru) & (np.abs(ax - ru) <= tau * (1 + np.abs(ru)))
    R = np.nonzero(rtl | rtu)[0]
    bR = np.where(rtl[R], rl[R], ru[R])
    Ad = A.toarray()
    AR = Ad[R]
    nF, nR = F.size, R.size
    K = np.zeros((nF + nR, nF + nR))
    K[:nF, :nF] = np.diag(q[F])
    K[:nF, nF:] = -AR[:, F].T
    K[nF:, :nF] = AR[:, F]
    rhs = np.concatenate([-c[F], bR - AR[:, bnd] @ xb[bnd]])
    sol, *_ = np.linalg.lstsq(K, rhs, rcond=None)
    x = xb.copy()
    x[F] = sol[:nF]
    y = np.zeros(A.shape[0])
    y[R] = sol[nF:]
    return x, y


def _kkt_solve(c, q, Ad, rl, ru, l, u, atl, atu, rtl, rtu):
    """Equality KKT system of an active set (lstsq: dependent rows/columns
    of degenerate LP parts get the minimum-norm solution)."""
    n = c.size
    fix = atl | atu
    xb = np.where(atl, l, np.where(atu, u, 0.0))
    F = np.nonzero(~fix)[0]
    R = np.nonzero(rtl | rtu)[0]
    bR = np.where(rtl[R], rl[R], ru[R])
    AR = Ad[R]
    nF, nR = F.size, R.size
    K = np.zeros((nF + nR, nF + nR))
    K[:nF, :nF] = np.diag(q[F])
    K[:nF, nF:] = -AR[:, F].T
    K[nF:, :nF] = AR[:, F]
    rhs = np.concatenate([-c[F], bR - AR[:, fix] @ xb[fix]])
    sol, *_ = np.linalg.lstsq(K, rhs, rcond=None)
    x = xb.copy()
    x[F] = sol[:nF]
    y = np.zeros(Ad.shape[0])
    y[R] = sol[nF:]
    return x, y


# scenarios with more lines than this avoid the dense paths (lstsq on the
# dense KKT matrix): farmer crops_multiplier 1000 has 21,001 lines
DENSE_MAX = 2000


def _pdas(x0, c, q, A, rl, ru, l, u, tau, kkt_tol, rounds=20):
    """Primal-dual active-set iterations from the active set of x0 (the same
    rule as the GPU polish): accepted when the clipped point passes the KKT
    check.  Returns (err, x, y) of the best point.  Large scenarios solve
    each active set's KKT system by the regularised sparse LU (_kkt_reg)."""
    large = A.shape[0] + A.shape[1] > DENSE_MAX
    Ad = sp.csr_matrix(A) if large else sp.csr_matrix(A).toarray()
    ax = Ad @ x0
    eq = np.isfinite(l) & (l == u)
    atl = eq | (np.isfinite(l) & (np.abs(x0 - l) <= tau * (1 + np.abs(l))))
    atu = ~atl & np.isfinite(u) & (np.abs(x0 - u) <= tau * (1 + np.abs(u)))
    req = np.isfinite(rl) & (rl == ru)
    rtl = req | (np.isfinite(rl) & (np.abs(ax - rl) <= tau * (1 + np.abs(rl))))
    rtu = ~rtl & np.isfinite(ru) & (np.abs(ax - ru) <= tau * (1 + np.abs(ru)))
    best = (np.inf, None, None)
    seen = set()
    for _ in range(rounds):
        key = (atl.tobytes(), atu.tobytes(), rtl.tobytes(), rtu.tobytes())
        if key in seen:
            break
        seen.add(key)
        if large:
            try:
                xu, y = _kkt_reg(c, q, Ad, rl, ru, l, u, atl, atu, rtl, rtu)
            except RuntimeError:  # singular factor
                break
        else:
            xu, y = _kkt_solve(c, q, Ad, rl, ru, l, u, atl, atu, rtl, rtu)
        x = np.minimum(np.maximum(xu, l), u)
        pv, dv = kkt_residual(x, y, c, q, A, rl, ru, l, u)
        err = max(pv, dv)
        if err < best[0]:
            best = (err, x, y)
        if err <= kkt_tol:
            break
        lam = q * xu + c - Ad.T @ y
        axu = Ad @ xu
        atl = eq | (np.isfinite(l) & (lam + (l - xu) > 0))
        atu = ~atl & np.isfinite(u) & (-lam + (xu - u) > 0)
        rtl = req | (np.isfinite(rl) & (y + (rl - axu) > 0))
        rtu = ~rtl & np.isfinite(ru) & (-y + (axu - ru) > 0)
    return best


def _checked_vertex(x, rowdual, c, q, A, rl, ru, l, u, kkt_tol):
    """HiGHS' simplex vertex with the row-dual sign that passes the KKT
    check (HiGHS reports d(obj)/d(activity); the oracle's y > 0 means a row
    at rl), or OracleSolveError when neither sign does."""
    best = None
    for y in (rowdual, -rowdual):
        err = max(kkt_residual(x, y, c, q, A, rl, ru, l, u))
        if best is None or err < best[0]:
            best = (err, y)
    if best[0] > kkt_tol:
        raise OracleSolveError(f"simplex vertex fails the KKT check: residual {best[0]:.3e}")
    return x, best[1], True


def solve_scenario(c, q, A, rl, ru, l, u, kkt_tol=1e-9):
    """Solve min 1/2 x'diag(q)x + c'x s.t. rl<=Ax<=ru, l<=x<=u exactly.

    Returns (x, y, feasible).  Raises OracleSolveError if no polished point
    passes the KKT check.
    """
    q = np.zeros_like(c) if q is None else np.asarray(q, dtype=np.float64)
    status, x, rowdual, _ = _highs_solve(c, q, A, rl, ru, l, u,
                                         time_limit=5.0 if np.any(q) else 20.0)
    name = str(status)
    if "Infeasible" in name or "Unbounded" in name:
        return None, None, False
    if "TimeLimit" in name and np.any(q):
        xc = _qp_by_cuts(c, q, A, rl, ru, l, u)
        if xc is None:
            raise OracleSolveError("HiGHS QP time limit and the cut fallback failed")
        best = (np.inf, None, None)
        if _last_basis is not None and _last_basis[0].size == c.size:
            bp = _basis_polish(c, q, A, rl, ru, l, u, kkt_tol)
            if bp is not None:
                best = bp
                if bp[0] <= kkt_tol:
                    return bp[1], bp[2], True
        for tau in (1e-6, 1e-5, 1e-7, 1e-4, 1e-8):
            err, xp, yp = _pdas(xc, c, q, A, rl, ru, l, u, tau, kkt_tol)
            if err < best[0]:
                best = (err, xp, yp)
            if err <= kkt_tol:
                return xp, yp, True
        raise OracleSolveError(f"QP cut fallback polish failed, best KKT residual {best[0]:.3e}")
    if "Optimal" not in name:
        raise OracleSolveError(f"HiGHS status {name}")
    # HiGHS row duals: d(obj)/d(row activity); our y = -rowdual? -> determine
    # the sign by the stationarity residual and keep the better one.
    best = None
    if np.any(q):
        # HiGHS' own QP point is sometimes already KKT-exact (sslp): keep it
        pv, dv = kkt_residual(x, rowdual, c, q, A, rl, ru, l, u)
        best = (max(pv, dv), x, rowdual)
        if best[0] <= kkt_tol:
            return x, rowdual, True
    if np.any(q) and A.shape[0] + A.shape[1] > 200:
        # larger prox-QPs (farmer crops_multiplier 100): the basis HiGHS ends
        # with names the active set; its KKT system solved exactly
        bp = _basis_polish(c, q, A, rl, ru, l, u, kkt_tol)
        if bp is not None:
            if bp[0] < best[0]:
                best = bp
            if bp[0] <= kkt_tol:
                return bp[1], bp[2], True
    large = A.shape[0] + A.shape[1] > DENSE_MAX
    if not np.any(q) and large:
        # a large LP's simplex vertex is exact to its tolerances (the dense
        # polish below is for small degenerate QP/LP cases): verified
        return _checked_vertex(x, rowdual, c, q, A, rl, ru, l, u, kkt_tol)
    for tau in (1e-7, 1e-8, 1e-6, 1e-9, 1e-5, 1e-10, 1e-4):
        if large:
            break
        xp, yp = _polish(x, c, q, A, rl, ru, l, u, tau)
        pv, dv = kkt_residual(xp, yp, c, q, A, rl, ru, l, u)
        err = max(pv, dv)
        if best is None or err < best[0]:
            best = (err, xp, yp)
        if err <= kkt_tol:
            return xp, yp, True
    if not np.any(q):
        # an LP vertex from simplex is already exact to its tolerances
        return _checked_vertex(x, rowdual, c, q, A, rl, ru, l, u, kkt_tol)
    # degenerate LP parts (many free columns without a prox term): the
    # tolerance guess of the active set is off -- primal-dual active-set
    # iterations from it, as the GPU polish does
    for tau in (1e-7, 1e-5, 1e-9):
        err, xp, yp = _pdas(x, c, q, A, rl, ru, l, u, tau, kkt_tol)
        if err < best[0]:
            best = (err, xp, yp)
        if err <= kkt_tol:
            return xp, yp, True
    raise OracleSolveError(f"QP polish failed, best KKT residual {best[0]:.3e}")
