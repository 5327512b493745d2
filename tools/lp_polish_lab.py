"""CPU lab (development tool: not product, not oracle) for the big path's
LP polish on farmer c=1000 (F4).  Restates, in numpy/scipy, the scaling
(big_scale_kernel), the restarted reflected-Halpern PDHG (solve_big) and the
PDAS LDL' polish (polish_big) closely enough to see why the Iter0 LP polish
fails, and to try changes before they go to the HIP kernels.

    python tools/lp_polish_lab.py [scen] [c] [variant]

The exact LP (HiGHS simplex through oracle.solve) is the yardstick.
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import models as om  # noqa: E402
from oracle.solve import solve_scenario  # noqa: E402


def scale(A):
    """big_scale_kernel: 10 Ruiz (inf-norm) sweeps + one Pock-Chambolle (l1)
    sweep, factors computed from the same state and then applied; step size
    from 64 power iterations on A~'A~."""
    A = sp.csr_matrix(A)
    m, n = A.shape
    dr = np.ones(m)
    dc = np.ones(n)
    absA = abs(A).tocsr()
    for sweep in range(11):
        As = sp.diags(dr) @ absA @ sp.diags(dc)
        if sweep < 10:
            rmax = np.asarray(As.max(axis=1).todense()).ravel()
            cmax = np.asarray(As.max(axis=0).todense()).ravel()
        else:
            rmax = np.asarray(As.sum(axis=1)).ravel()
            cmax = np.asarray(As.sum(axis=0)).ravel()
        dr *= np.where(rmax > 0, 1 / np.sqrt(np.where(rmax > 0, rmax, 1)), 1.0)
        dc *= np.where(cmax > 0, 1 / np.sqrt(np.where(cmax > 0, cmax, 1)), 1.0)
    As = (sp.diags(dr) @ A @ sp.diags(dc)).tocsr()
    v = np.ones(n)
    est = 1.0
    for _ in range(64):
        w = As.T @ (As @ v)
        nrm = np.linalg.norm(w)
        est = np.sqrt(nrm)
        v = w / nrm if nrm > 0 else w * 0
    sn = min(1.0, 1.02 * est)
    if not sn > 1e-12:
        sn = 1.0
    return As, dr, dc, 0.995 / sn


class Scaled:
    def __init__(self, sc, g=None, q=None):
        self.A, self.dr, self.dc, self.eta = scale(sc.A)
        self.AT = self.A.T.tocsr()
        dc, dr = self.dc, self.dr
        g = sc.c if g is None else g
        q = np.zeros_like(sc.c) if q is None else q
        self.G = g * dc
        self.Q = q * dc * dc
        self.L = sc.l / dc
        self.U = sc.u / dc
        self.RL = sc.rl * dr
        self.RU = sc.ru * dr
        self.n, self.m = sc.A.shape[1], sc.A.shape[0]

    def kkt(self, xs, ys, axs=None):
        """kkt_rel of the scaled point (xs, ys): ep, ed, eg, pobj, dobj."""
        if axs is None:
            axs = self.A @ xs
        dc, dr = self.dc, self.dr
        aty = self.AT @ ys
        lam = (self.Q * xs + self.G - aty) / dc
        xu = xs * dc
        lu, uu = self.L * dc, self.U * dc
        lp = np.where(np.isfinite(lu), np.maximum(lam, 0), 0)
        lm = np.where(np.isfinite(uu), np.minimum(lam, 0), 0)
        rd = lam - lp - lm
        qx = self.Q / dc / dc
        gu = self.G / dc
        axu = axs / dr
        rlu, ruu = self.RL / dr, self.RU / dr
        rp = axu - np.clip(axu, rlu, ruu)
        yu = ys * dr
        bad = ((yu > 0) & ~np.isfinite(rlu)) | ((yu < 0) & ~np.isfinite(ruu))
        v1 = np.sum(rd * rd) + np.sum(yu[bad] ** 2)
        yu = np.where(bad, 0.0, yu)
        pobj = np.sum(0.5 * qx * xu * xu + gu * xu)
        dobj = (np.sum(-0.5 * qx * xu * xu) + np.sum(np.where(lp > 0, lp * np.where(np.isfinite(lu), lu, 0), 0))
                + np.sum(np.where(lm < 0, lm * np.where(np.isfinite(uu), uu, 0), 0))
                + np.sum(np.where(yu > 0, yu * np.where(np.isfinite(rlu), rlu, 0), 0))
                + np.sum(np.where(yu < 0, yu * np.where(np.isfinite(ruu), ruu, 0), 0)))
        b2 = np.sum(np.where(np.isfinite(rlu), rlu, 0) ** 2)
        ep = np.sqrt(np.sum(rp * rp)) / (1 + np.sqrt(b2))
        ed = np.sqrt(v1) / (1 + np.sqrt(np.sum(gu * gu)))
        eg = abs(pobj - dobj) / (1 + abs(pobj) + abs(dobj))
        return ep, ed, eg, pobj, dobj


def pdhg(P, x, y, exit_err, maxit=200000, chk=64, gam=1.0, omega=None, span=1e6, verbose=False, callback=None):
    """solve_big's PDHG from the scaled point (x, y): returns the trial point
    whose max KKT error is <= exit_err (or the last one), steps, error."""
    A, AT = P.A, P.AT
    x = np.clip(x, P.L, P.U)
    y = y.copy()
    y = np.where(~np.isfinite(P.RL), np.minimum(y, 0), y)
    y = np.where(~np.isfinite(P.RU), np.maximum(y, 0), y)
    bl = np.where(np.isfinite(P.RL), P.RL, 0)
    bu = np.where(np.isfinite(P.RU), P.RU, 0)
    bsq = np.sum(bl * bl + np.where(np.isfinite(P.RL), 0, bu * bu))
    gn, bn = np.linalg.norm(P.G), np.sqrt(bsq)
    omega0 = gn / bn if (gn > 1e-10 and bn > 1e-10) else 1.0
    om_ = omega0 if omega is None else np.clip(omega, omega0 / span, omega0 * span)
    eta = P.eta

    def steps(om_):
        tau = eta / om_
        return tau, eta * om_, 1.0 / (1.0 + tau * P.Q)
    tau, sig, iq = steps(om_)
    X, Z0X, XN = x.copy(), x.copy(), x.copy()
    Y, Z0Y = y.copy(), y.copy()
    AX = A @ x
    AZ0 = AX.copy()
    k = 0
    r_restart = r_prev = -1.0
    err = np.inf
    for it in range(maxit):
        cb = 1.0 / (k + 2)
        ca = (k + 1) * cb
        check = (it % chk) == 0 or it == maxit - 1
        aty = AT @ Y
        xn = np.clip((X - tau * (P.G - aty)) * iq, P.L, P.U)
        dxx = np.sum((xn - X) ** 2)
        X = ca * ((1 + gam) * xn - gam * X) + cb * Z0X
        axn = A @ xn
        v = Y - sig * (2 * axn - AX)
        yn = np.maximum(v + sig * P.RL, 0) + np.minimum(v + sig * P.RU, 0)
        dyy = np.sum((yn - Y) ** 2)
        Y = ca * ((1 + gam) * yn - gam * Y) + cb * Z0Y
        AX = ca * ((1 + gam) * axn - gam * AX) + cb * AZ0
        k += 1
        if not check:
            continue
        ep, ed, eg, _, _ = P.kkt(xn, yn, axn)
        err = max(ep, ed, eg)
        if verbose and it % 4096 == 0:
            print(f"    pdhg {it}: ep {ep:.2e} ed {ed:.2e} eg {eg:.2e} omega {om_:.3e}")
        if err <= exit_err:
            return xn, yn, it + 1, err, om_
        if callback is not None and callback(it + 1, xn, yn, err):
            return xn, yn, it + 1, err, om_
        r = np.sqrt(om_ * dxx + dyy / om_)
        restart = False
        if r_restart < 0:
            r_restart = r
        else:
            restart = r <= 0.2 * r_restart or (r <= 0.8 * r_restart and r > r_prev) or k >= 0.36 * (it + 1)
        r_prev = r
        reset = it > 0 and ((it + 1) % 8192) < chk and (om_ > span * omega0 or om_ * span < omega0)
        if reset:
            om_ = omega0
            restart = True
        elif restart:
            dx, dy = np.linalg.norm(xn - Z0X), np.linalg.norm(yn - Z0Y)
            if dx > 1e-12 and dy > 1e-12:
                om_ = np.sqrt(dy / dx * om_)
        if restart:
            tau, sig, iq = steps(om_)
            X, Z0X = xn.copy(), xn.copy()
            Y, Z0Y = yn.copy(), yn.copy()
            AX, AZ0 = axn.copy(), axn.copy()
            k = 0
            r_restart = r
    return xn, yn, maxit, err, om_


def polish(P, xs, ys, th, tol=1e-9, rounds=6, delta=1e-7, refine=8, refine_tol=1e-12, pin=True,
           verbose=True, variant=None, exact=None):
    """polish_big restated: classify (xs, ys) at threshold th, then PDAS
    rounds of the regularised KKT solve with refinement; returns (ok, x, y)."""
    variant = variant or {}
    A, AT = P.A, P.AT
    n, m = P.n, P.m
    L, U, RL, RU, G, Q = P.L, P.U, P.RL, P.RU, P.G, P.Q
    Ac = A.tocoo()
    CC = np.zeros(n, dtype=int)
    CC[L == U] = 1
    atl = np.isfinite(L) & (xs - L <= th * (1 + np.abs(L)))
    atu = np.isfinite(U) & (U - xs <= th * (1 + np.abs(U)))
    CC = np.where(L == U, 1, np.where(atl, 1, np.where(atu, 2, 0)))
    ym = np.max(np.abs(ys))
    RC = np.where(RL == RU, 1, np.where(np.isfinite(RL) & (ys > th * ym), 1,
                                        np.where(np.isfinite(RU) & (ys < -th * ym), 2, 0)))
    if variant.get("init") == "pdas":  # the PDAS rule on the trial point itself
        axs = A @ xs
        lam0 = Q * xs + G - AT @ ys
        CC = np.where(L == U, 1, np.where(np.isfinite(L) & (lam0 + (L - xs) > 0), 1,
                                          np.where(np.isfinite(U) & (-lam0 + (xs - U) > 0), 2, 0)))
        RC = np.where(RL == RU, 1, np.where(np.isfinite(RL) & (ys + (RL - axs) > 0), 1,
                                            np.where(np.isfinite(RU) & (-ys + (axs - RU) > 0), 2, 0)))
    YFX = ys.copy()
    for rnd in range(rounds):
        free = CC == 0
        act = RC != 0
        # pinned rows: active with no free column
        nfree_row = np.asarray(sp.csr_matrix((free[Ac.col].astype(float), (Ac.row, Ac.col)),
                                             shape=(m, n)).sum(axis=1)).ravel()
        PIN = act & (nfree_row == 0) if pin else np.zeros(m, bool)
        PX = np.where(CC == 1, L, np.where(CC == 2, U, 0.0))
        RHX = np.where(free, -G, PX)
        ax_fixed = A @ PX
        yproj = np.where(~np.isfinite(RL), np.minimum(YFX, 0), YFX)
        yproj = np.where(~np.isfinite(RU), np.maximum(yproj, 0), yproj)
        bnd = np.where(RC == 1, RL, RU)
        RHY = np.where(act, np.where(PIN, -yproj, -(np.where(act, bnd, 0) - ax_fixed)), 0.0)
        # T (unregularised) and Treg
        keep = free[Ac.col] & act[Ac.row] & ~PIN[Ac.row]
        ri, cj, av = Ac.row[keep], Ac.col[keep], Ac.data[keep]
        Hd = np.where(free, Q, 1.0)
        Gd = np.where(act & ~PIN, 0.0, -1.0)
        off = sp.coo_matrix((np.concatenate([-av, -av]), (np.concatenate([cj, n + ri]),
                                                          np.concatenate([n + ri, cj]))), shape=(n + m, n + m))
        T = (off + sp.diags(np.concatenate([Hd, Gd]))).tocsc()
        Treg = (T + sp.diags(np.concatenate([np.where(free, delta, 0.0),
                                             np.where(act & ~PIN, -delta, 0.0)]))).tocsc()
        lu = spla.splu(Treg, permc_spec="MMD_AT_PLUS_A", diag_pivot_thresh=0.0,
                       options=dict(SymmetricMode=True))
        rhs = np.concatenate([RHX, RHY])
        z = np.zeros(n + m)
        if variant.get("z0") == "warm":  # refinement from the trial point
            z = np.concatenate([np.where(free, xs if rnd == 0 else ZX, RHX), np.where(act, ys if rnd == 0 else ZY, 0.0)])
        hist = []
        ref_ok = False
        for itr in range(refine):
            r = rhs - T @ z
            rc = np.abs(r) / (1 + np.abs(rhs))
            hist.append(rc.max())
            if itr > 0 and not rc.max() > min(refine_tol, 1e-3 * tol):
                ref_ok = True
                break
            if variant.get("stag") and itr > 1 and rc.max() > 0.5 * hist[-2]:
                break  # stagnating: an inconsistent system; stop before it blows up
            z = z + lu.solve(r)
        if not ref_ok:
            r = rhs - T @ z
            hist.append((np.abs(r) / (1 + np.abs(rhs))).max())
            ref_ok = hist[-1] <= min(refine_tol, 1e-3 * tol)
        ZX, ZY = z[:n], z[n:]
        PXc = np.clip(ZX, L, U)
        ep, ed, eg, pobj, dobj = P.kkt(PXc, ZY)
        lam = Q * PXc + G - AT @ ZY
        nclip = int(np.sum(PXc != ZX))
        info = (f"  round {rnd}: free {free.sum()} act {act.sum()} pinned {PIN.sum()} | refine "
                + " ".join(f"{h:.0e}" for h in hist) + f" | ep {ep:.2e} ed {ed:.2e} eg {eg:.2e} clipped {nclip}")
        if exact is not None:
            xe, ce, re_ = exact
            info += f" | col mismatch {np.sum(CC != ce)} row mismatch {np.sum((RC != 0) != (re_ != 0))}"
        if verbose:
            print(info)
        if ep <= tol and ed <= tol and eg <= tol:
            return True, PXc, ZY, rnd + 1
        # re-classification from the unclipped point
        axu = A @ ZX
        lamu = lam + Q * (ZX - PXc)
        cw = variant.get("cw", 1.0)
        if "ci" in variant and not ref_ok:
            cw = float(variant["ci"])  # an inconsistent system: trust the residual's sign more
        cs = np.where(L == U, 1, np.where(np.isfinite(L) & (lamu + cw * (L - ZX) > 0), 1,
                                          np.where(np.isfinite(U) & (-lamu + cw * (ZX - U) > 0), 2, 0)))
        zy = ZY.copy()
        rs = np.where(RL == RU, 1, np.where(np.isfinite(RL) & (zy + cw * (RL - axu) > 0), 1,
                                            np.where(np.isfinite(RU) & (-zy + cw * (axu - RU) > 0), 2, 0)))
        changed = int(np.sum(cs != CC) + np.sum(rs != RC))
        if verbose:
            print(f"     changed {changed} (cols {np.sum(cs != CC)}, rows {np.sum(rs != RC)})")
            if exact is not None and changed < 40:
                for j in np.nonzero(cs != CC)[0]:
                    print(f"       col {j} {CC[j]}->{cs[j]} exact {exact[1][j]} zx {ZX[j]:.4g} lam {lamu[j]:.3g} L {L[j]:.3g} U {U[j]:.3g}")
                for i in np.nonzero(rs != RC)[0]:
                    print(f"       row {i} {RC[i]}->{rs[i]} exact {exact[2][i]} zy {ZY[i]:.4g} slack {axu[i] - (RL[i] if np.isfinite(RL[i]) else RU[i]):.3g}")
        CC, RC, YFX = cs, rs, zy
        if changed == 0:
            return False, PXc, ZY, rnd + 1
    return False, PXc, ZY, rounds


def main():
    sn = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    c = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    variant = dict(kv.split("=") for kv in sys.argv[3:])
    sc = om.farmer(f"scen{sn}", c)
    t = time.time()
    P = Scaled(sc)
    print(f"scen{sn} c={c}: n={P.n} m={P.m} eta={P.eta:.4f} scaling {time.time() - t:.1f}s")
    t = time.time()
    q = np.zeros(P.n)
    xe, ye, feas = solve_scenario(sc.c, q, sc.A, sc.rl, sc.ru, sc.l, sc.u)
    xes, yes_ = xe / P.dc, ye / P.dr
    print(f"HiGHS: obj {sc.c @ xe:.10e} ({time.time() - t:.1f}s); scaled KKT {P.kkt(xes, yes_)[:3]}")
    the = 1e-9
    ce = np.where(P.L == P.U, 1, np.where(np.isfinite(P.L) & (xes - P.L <= the * (1 + np.abs(P.L))), 1,
                                          np.where(np.isfinite(P.U) & (P.U - xes <= the * (1 + np.abs(P.U))), 2, 0)))
    axe = P.A @ xes
    re_ = np.where(np.isfinite(P.RL) & (np.abs(axe - P.RL) <= 1e-9 * (1 + np.abs(P.RL))), 1,
                   np.where(np.isfinite(P.RU) & (np.abs(axe - P.RU) <= 1e-9 * (1 + np.abs(P.RU))), 2, 0))
    print(f"exact: free cols {np.sum(ce == 0)}, tight rows {np.sum(re_ != 0)}, y!=0 rows {np.sum(yes_ != 0)}")
    x = np.zeros(P.n)
    y = np.zeros(P.m)
    om_ = None
    steps = 0
    for exit_err in (1e-4, 1e-6, 1e-8):
        t = time.time()
        x, y, it, err, om_ = pdhg(P, x, y, exit_err, omega=om_)
        steps += it
        print(f"PDHG to {exit_err:.0e}: {it} steps (total {steps}), err {err:.2e} ({time.time() - t:.1f}s); "
              f"|x-x*|inf {np.abs(x * P.dc - xe).max():.3e}")
        th = min(np.sqrt(max(err, 0.0)), 1e-3)
        ok, xp, yp, rnds = polish(P, x, y, th, exact=(xes, ce, re_), variant=variant)
        print(f"  polish th={th:.1e}: ok={ok} rounds {rnds}" +
              (f" obj {sc.c @ (xp * P.dc):.10e}" if ok else ""))
        if ok:
            break


if __name__ == "__main__":
    main()


def polish_prox(P, xs, ys, tol=1e-9, deltas=(1e-2, 1e-3, 1e-4, 1e-5, 1e-6, 1e-7, 1e-7, 1e-7), refine=3,
                verbose=True, exact=None, pin=True):
    """Proximal semismooth-Newton variant: each round classifies the current
    point by the PDAS rule, then takes regularised KKT steps anchored at the
    current point with delta from a decreasing schedule (an inconsistent
    active set cannot blow the step up beyond |residual| / delta)."""
    A, AT = P.A, P.AT
    n, m = P.n, P.m
    L, U, RL, RU, G, Q = P.L, P.U, P.RL, P.RU, P.G, P.Q
    Ac = A.tocoo()
    X, Y = xs.copy(), ys.copy()
    for rnd, delta in enumerate(deltas):
        ax = A @ X
        lam = Q * X + G - AT @ Y
        CC = np.where(L == U, 1, np.where(np.isfinite(L) & (lam + (L - X) > 0), 1,
                                          np.where(np.isfinite(U) & (-lam + (X - U) > 0), 2, 0)))
        RC = np.where(RL == RU, 1, np.where(np.isfinite(RL) & (Y + (RL - ax) > 0), 1,
                                            np.where(np.isfinite(RU) & (-Y + (ax - RU) > 0), 2, 0)))
        free = CC == 0
        act = RC != 0
        nfree_row = np.bincount(Ac.row, weights=free[Ac.col].astype(float), minlength=m)
        PIN = act & (nfree_row == 0) if pin else np.zeros(m, bool)
        PX = np.where(CC == 1, L, np.where(CC == 2, U, 0.0))
        RHX = np.where(free, -G, PX)
        ax_fixed = A @ PX
        yproj = np.where(~np.isfinite(RL), np.minimum(Y, 0), Y)
        yproj = np.where(~np.isfinite(RU), np.maximum(yproj, 0), yproj)
        bnd = np.where(RC == 1, RL, RU)
        RHY = np.where(act, np.where(PIN, -yproj, -(np.where(act, bnd, 0) - ax_fixed)), 0.0)
        keep = free[Ac.col] & act[Ac.row] & ~PIN[Ac.row]
        ri, cj, av = Ac.row[keep], Ac.col[keep], Ac.data[keep]
        Hd = np.where(free, Q, 1.0)
        Gd = np.where(act & ~PIN, 0.0, -1.0)
        off = sp.coo_matrix((np.concatenate([-av, -av]), (np.concatenate([cj, n + ri]),
                                                          np.concatenate([n + ri, cj]))), shape=(n + m, n + m))
        T = (off + sp.diags(np.concatenate([Hd, Gd]))).tocsc()
        Treg = (T + sp.diags(np.concatenate([np.where(free, delta, 0.0),
                                             np.where(act & ~PIN, -delta, 0.0)]))).tocsc()
        lu = spla.splu(Treg, permc_spec="MMD_AT_PLUS_A", diag_pivot_thresh=0.0, options=dict(SymmetricMode=True))
        rhs = np.concatenate([RHX, RHY])
        z = np.concatenate([np.where(free, X, PX), np.where(act, Y, 0.0)])
        hist = []
        for itr in range(refine):
            r = rhs - T @ z
            hist.append((np.abs(r) / (1 + np.abs(rhs))).max())
            if hist[-1] <= 1e-3 * tol:
                break
            z = z + lu.solve(r)
        r = rhs - T @ z
        hist.append((np.abs(r) / (1 + np.abs(rhs))).max())
        X, Y = z[:n], z[n:]
        Xc = np.clip(X, L, U)
        ep, ed, eg, pobj, dobj = P.kkt(Xc, Y)
        info = (f"  prox round {rnd} d={delta:.0e}: free {free.sum()} act {act.sum()} pinned {PIN.sum()} | res "
                + " ".join(f"{h:.0e}" for h in hist) + f" | ep {ep:.2e} ed {ed:.2e} eg {eg:.2e}")
        if exact is not None:
            info += f" | col mismatch {np.sum(CC != exact[1])} row mismatch {np.sum((RC != 0) != (exact[2] != 0))}"
        if verbose:
            print(info)
        if ep <= tol and ed <= tol and eg <= tol:
            return True, Xc, Y, rnd + 1
    return False, np.clip(X, L, U), Y, len(deltas)


def _kkt_system(P, CC, RC, Y, delta, pin=True):
    """The active set's KKT matrix T, its regularisation and the rhs (as polish)."""
    A = P.A
    n, m = P.n, P.m
    L, U, RL, RU, G, Q = P.L, P.U, P.RL, P.RU, P.G, P.Q
    Ac = A.tocoo()
    free = CC == 0
    act = RC != 0
    nfree_row = np.bincount(Ac.row, weights=free[Ac.col].astype(float), minlength=m)
    PIN = act & (nfree_row == 0) if pin else np.zeros(m, bool)
    PX = np.where(CC == 1, L, np.where(CC == 2, U, 0.0))
    RHX = np.where(free, -G, PX)
    ax_fixed = A @ PX
    yproj = np.where(~np.isfinite(RL), np.minimum(Y, 0), Y)
    yproj = np.where(~np.isfinite(RU), np.maximum(yproj, 0), yproj)
    bnd = np.where(RC == 1, RL, RU)
    RHY = np.where(act, np.where(PIN, -yproj, -(np.where(act, bnd, 0) - ax_fixed)), 0.0)
    keep = free[Ac.col] & act[Ac.row] & ~PIN[Ac.row]
    ri, cj, av = Ac.row[keep], Ac.col[keep], Ac.data[keep]
    Hd = np.where(free, Q, 1.0)
    Gd = np.where(act & ~PIN, 0.0, -1.0)
    off = sp.coo_matrix((np.concatenate([-av, -av]), (np.concatenate([cj, n + ri]),
                                                      np.concatenate([n + ri, cj]))), shape=(n + m, n + m))
    T = (off + sp.diags(np.concatenate([Hd, Gd]))).tocsc()
    Treg = (T + sp.diags(np.concatenate([np.where(free, delta, 0.0),
                                         np.where(act & ~PIN, -delta, 0.0)]))).tocsc()
    return T, Treg, np.concatenate([RHX, RHY]), PX, PIN


def polish_rt(P, xs, ys, tol=1e-9, rounds=12, delta=1e-7, refine=4, verbose=True, exact=None, enter=0.5, act_tol=0.0):
    """PDAS with a ratio test: the regularised KKT step from the current point
    is cut where a free column reaches a bound or an active row's multiplier
    changes sign (those entries change class); a full step re-classifies by
    the PDAS sign rule.  An inconsistent active set (a step along a null
    direction of the active set's matrix, 1/delta long) becomes a simplex-like
    move to the first blocking bound instead of a blow-up."""
    A, AT = P.A, P.AT
    n, m = P.n, P.m
    L, U, RL, RU, G, Q = P.L, P.U, P.RL, P.RU, P.G, P.Q
    ax = A @ xs
    lam = Q * xs + G - AT @ ys
    CC = np.where(L == U, 1, np.where(np.isfinite(L) & (lam + (L - xs) > 0), 1,
                                      np.where(np.isfinite(U) & (-lam + (xs - U) > 0), 2, 0)))
    RC = np.where(RL == RU, 1, np.where(np.isfinite(RL) & (ys + (RL - ax) > 0), 1,
                                        np.where(np.isfinite(RU) & (-ys + (ax - RU) > 0), 2, 0)))
    X = np.where(CC == 1, L, np.where(CC == 2, U, xs))
    Y = np.where(RC != 0, ys, 0.0)
    for rnd in range(rounds):
        T, Treg, rhs, PX, PIN = _kkt_system(P, CC, RC, Y, delta)
        free, act = CC == 0, RC != 0
        X = np.where(free, X, PX)
        Y = np.where(act, Y, 0.0)
        lu = spla.splu(Treg, permc_spec="MMD_AT_PLUS_A", diag_pivot_thresh=0.0, options=dict(SymmetricMode=True))
        z0 = np.concatenate([X, Y])
        z = z0.copy()
        hist = []
        for itr in range(refine):
            r = rhs - T @ z
            hist.append((np.abs(r) / (1 + np.abs(rhs))).max())
            if hist[-1] <= 1e-3 * tol or (itr > 1 and hist[-1] > 0.5 * hist[-2]):
                break
            z = z + lu.solve(r)
        d = z - z0
        dx, dy = d[:n], d[n:]
        # ratio test: free columns leaving [L, U]; active (non-pinned) rows' multipliers changing sign
        tcol = np.full(n, np.inf)
        up = free & (dx > 0) & np.isfinite(U)
        dn = free & (dx < 0) & np.isfinite(L)
        tcol[up] = (U[up] - X[up]) / dx[up]
        tcol[dn] = (L[dn] - X[dn]) / dx[dn]
        trow = np.full(m, np.inf)
        two = RL == RU
        r1 = act & ~two & ~PIN & (RC == 1) & (dy < 0)
        r2 = act & ~two & ~PIN & (RC == 2) & (dy > 0)
        trow[r1] = -Y[r1] / dy[r1]
        trow[r2] = -Y[r2] / dy[r2]
        t = min(1.0, tcol.min(initial=np.inf), trow.min(initial=np.inf))
        t = max(t, 0.0)
        X = X + t * dx
        Y = Y + t * dy
        Xc = np.clip(X, L, U)
        ep, ed, eg, pobj, dobj = P.kkt(Xc, Y)
        nbc = int(np.sum(tcol <= t * (1 + 1e-12))) if t < 1 else 0
        nbr = int(np.sum(trow <= t * (1 + 1e-12))) if t < 1 else 0
        info = (f"  rt round {rnd}: free {free.sum()} act {act.sum()} pinned {PIN.sum()} | res "
                + " ".join(f"{h:.0e}" for h in hist) + f" | t {t:.3g} blocks {nbc}c/{nbr}r"
                f" | ep {ep:.2e} ed {ed:.2e} eg {eg:.2e}")
        if exact is not None:
            info += f" | col mismatch {np.sum(CC != exact[1])} row mismatch {np.sum((RC != 0) != (exact[2] != 0))}"
        if verbose:
            print(info)
        if ep <= tol and ed <= tol and eg <= tol:
            return True, Xc, Y, rnd + 1
        if t < 1.0:
            tt = t * (1 + 1e-12)
            bc = np.nonzero(tcol <= tt)[0]
            for j in bc:
                CC[j] = 2 if dx[j] > 0 else 1
            br = np.nonzero(trow <= tt)[0]
            RC[br] = 0
            Y[br] = 0.0
        else:
            # full step: the PDAS sign rule on fixed columns / inactive rows
            lam = Q * Xc + G - AT @ Y
            axc = A @ X
            rel_c = (CC == 1) & (lam < 0) & (L != U) | (CC == 2) & (lam > 0) & (L != U)
            if enter < 1 and rel_c.any():  # within a factor of the largest violation
                viol = np.where(rel_c, np.abs(lam), 0.0)
                rel_c = viol >= enter * viol.max()
            elif rel_c.sum() > enter:  # the most violated few only (an unreliable dual frees thousands)
                viol = np.where(rel_c, np.abs(lam), 0.0)
                keep = np.argsort(-viol)[:enter]
                rel_c = np.zeros(n, bool)
                rel_c[keep] = True
            CC[rel_c] = 0
            ptol = act_tol * (1 + np.abs(np.where(np.isfinite(RL), RL, 0)))
            ac1 = (RC == 0) & np.isfinite(RL) & (axc < RL - ptol)
            ptol = act_tol * (1 + np.abs(np.where(np.isfinite(RU), RU, 0)))
            ac2 = (RC == 0) & np.isfinite(RU) & (axc > RU + ptol)
            RC[ac1] = 1
            RC[ac2] = 2
            if verbose:
                print(f"     full step: freed {rel_c.sum()} cols, activated {ac1.sum() + ac2.sum()} rows")
            if not (rel_c.any() or ac1.any() or ac2.any()):
                return False, Xc, Y, rnd + 1
    return False, np.clip(X, L, U), Y, rounds
