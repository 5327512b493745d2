"""Lab (not product): a primal-dual interior-point method (Mehrotra
predictor-corrector) for one scenario's LP / prox-QP on the supernodal
quasi-definite LDL' of the device (CPU replay: libsuper_cpu.so), to settle
the algorithm before writing it as a HIP kernel.

    python tools/ipm_lab/ipm_lab.py uc 3          # UC Scenario1..3 LPs (+ a prox-QP)
"""
import ctypes
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy_amd"))
sys.path.insert(0, ROOT)

lib = ctypes.CDLL(os.path.join(HERE, "libsuper_cpu.so"))
lib.sc_create.restype = ctypes.c_void_p
lib.sc_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
lib.sc_factor.restype = ctypes.c_long
lib.sc_factor.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                          ctypes.c_double]
lib.sc_solve.argtypes = [ctypes.c_void_p, ctypes.c_void_p]


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class Factor:
    def __init__(self, n, m, rp, ci):
        self.rp = np.ascontiguousarray(rp, dtype=np.int32)
        self.ci = np.ascontiguousarray(ci, dtype=np.int32)
        info = np.zeros(8, dtype=np.int64)
        self.h = lib.sc_create(n, m, ptr(self.rp), ptr(self.ci), ptr(info))
        assert self.h
        self.info = info
        self.n, self.m = n, m

    def factor(self, diag, aval, cmask, rmask, delta):
        self.diag = np.ascontiguousarray(diag)
        return lib.sc_factor(self.h, ptr(self.diag), ptr(np.ascontiguousarray(aval)),
                             ptr(np.ascontiguousarray(cmask, dtype=np.int32)),
                             ptr(np.ascontiguousarray(rmask, dtype=np.int32)), delta)

    def solve(self, rhs):
        r = np.ascontiguousarray(rhs, dtype=np.float64).copy()
        lib.sc_solve(self.h, ptr(r))
        return r


def ruiz_pc(A, iters=10):
    """Ruiz equilibration then Pock-Chambolle (alpha = 1): A~ = Dr A Dc."""
    A = sp.csr_matrix(A, copy=True)
    m, n = A.shape
    dr = np.ones(m)
    dc = np.ones(n)
    for _ in range(iters):
        B = sp.diags(dr) @ A @ sp.diags(dc)
        rn = np.sqrt(abs(B).max(axis=1).toarray().ravel())
        cn = np.sqrt(abs(B).max(axis=0).toarray().ravel())
        dr /= np.where(rn > 0, rn, 1.0)
        dc /= np.where(cn > 0, cn, 1.0)
    B = abs(sp.diags(dr) @ A @ sp.diags(dc))
    rs = np.sqrt(np.asarray(B.sum(axis=1)).ravel())
    cs = np.sqrt(np.asarray(B.sum(axis=0)).ravel())
    dr /= np.where(rs > 0, rs, 1.0)
    dc /= np.where(cs > 0, cs, 1.0)
    return dr, dc


def kkt_rel(x, y, g, q, A, rl, ru, l, u):
    """The product's acceptance measure (phgpu.hip kkt_terms_col / _row /
    kkt_rel), unscaled."""
    lam = q * x + g - A.T @ y
    lp = np.where(np.isfinite(l), np.maximum(lam, 0), 0)
    lm = np.where(np.isfinite(u), np.minimum(lam, 0), 0)
    rd = lam - lp - lm
    ax = A @ x
    rp = ax - np.clip(ax, rl, ru)
    yy = y.copy()
    bad = ((yy > 0) & ~np.isfinite(rl)) | ((yy < 0) & ~np.isfinite(ru))
    rdr = np.sum(yy[bad] ** 2)
    yy[bad] = 0
    pobj = 0.5 * np.sum(q * x * x) + g @ x
    dobj = (-0.5 * np.sum(q * x * x) + np.sum(np.where(lp > 0, lp * np.where(np.isfinite(l), l, 0), 0))
            + np.sum(np.where(lm < 0, lm * np.where(np.isfinite(u), u, 0), 0))
            + np.sum(np.where(yy > 0, yy * np.where(np.isfinite(rl), rl, 0), 0))
            + np.sum(np.where(yy < 0, yy * np.where(np.isfinite(ru), ru, 0), 0)))
    bn = np.sqrt(np.sum(np.where(np.isfinite(rl), rl, 0) ** 2))
    gn = np.sqrt(np.sum(g * g))
    ep = np.sqrt(np.sum(rp * rp)) / (1 + bn)
    ed = np.sqrt(np.sum(rd * rd) + rdr) / (1 + gn)
    eg = abs(pobj - dobj) / (1 + abs(pobj) + abs(dobj))
    return ep, ed, eg, pobj, dobj


def ipm(F, A, g, q, l, u, rl, ru, dr, dc, tol=1e-9, maxit=200, delta=1e-9, refine=3, verbose=True,
        x0=None, y0=None, mu0=None, cs_mode='max', push=1.0, eta_max=0.9999, zinit=0.0, sigmax=1e9, same_step=False, center_fb=0.0, relax=0.0):
    """Mehrotra predictor-corrector in the scaled space; A (csr, unscaled),
    data unscaled; returns unscaled x, y and the measure."""
    n, m = A.shape[1], A.shape[0]
    if relax > 0:
        # widen every inequality bound by relax (absolute, unscaled): an
        # interior for implied equalities of several rows
        fix0 = l == u
        l = np.where(fix0, l, l - relax)
        u = np.where(fix0, u, u + relax)
        eq0 = rl == ru
        rl = np.where(eq0, rl, rl - relax)
        ru = np.where(eq0, ru, ru + relax)
    As = sp.csr_matrix(sp.diags(dr) @ A @ sp.diags(dc))
    AsT = sp.csr_matrix(As.T)
    gs = g * dc
    qs = q * dc * dc
    # cost scaling: the scaled objective's largest coefficient 1 (the
    # multipliers come back times cs)
    ag = np.abs(gs[gs != 0])
    if cs_mode == 'max':
        cs = max(1.0, np.max(np.abs(gs)), np.max(qs, initial=0.0))
    elif cs_mode == 'geo':
        cs = float(np.exp(np.mean(np.log(ag)))) if ag.size else 1.0
    elif cs_mode == 'rms':
        cs = float(np.sqrt(np.mean(ag ** 2))) if ag.size else 1.0
    else:
        cs = 1.0
    if verbose:
        print('   cost scale', cs, 'max|gs|', np.max(np.abs(gs)))
    gs = gs / cs
    qs = qs / cs
    ls, us = l / dc, u / dc
    rls, rus = rl * dr, ru * dr
    # presolve: forcing rows (their activity bound equals the row bound: every
    # column at the bound that attains it) -> columns fixed, row dropped (its
    # multiplier set after the solve, postsolve below)
    forced = np.zeros(m, dtype=np.int8)  # +1: at rl (maxact), -1: at ru (minact)
    ls, us = ls.copy(), us.copy()
    rows_of = np.repeat(np.arange(m), np.diff(As.indptr))
    for _pass in range(40):
        a = As.data
        lo_c, hi_c = ls[As.indices], us[As.indices]
        with np.errstate(invalid='ignore'):
            tmin = np.where(a > 0, a * lo_c, np.where(a < 0, a * hi_c, 0.0))
            tmax = np.where(a > 0, a * hi_c, np.where(a < 0, a * lo_c, 0.0))
        minact = np.add.reduceat(tmin, As.indptr[:-1]) if As.nnz else np.zeros(m)
        maxact = np.add.reduceat(tmax, As.indptr[:-1]) if As.nnz else np.zeros(m)
        tolr = 1e-12 * (1 + np.abs(rls))
        fr_l = (forced == 0) & np.isfinite(rls) & np.isfinite(maxact) & (maxact <= rls + tolr)
        fr_u = (forced == 0) & np.isfinite(rus) & np.isfinite(minact) & (minact >= rus - 1e-12 * (1 + np.abs(rus)))
        if not (fr_l.any() or fr_u.any()):
            break
        print('presolve pass', _pass, fr_l.sum(), fr_u.sum())
        forced[fr_l] = 1
        forced[fr_u & ~fr_l] = -1
        for i in np.nonzero(fr_l | fr_u)[0]:
            sl = slice(As.indptr[i], As.indptr[i + 1])
            for j, aij in zip(As.indices[sl], As.data[sl]):
                if aij == 0:
                    continue
                up_side = (aij > 0) == (forced[i] == 1)
                v = us[j] if up_side else ls[j]
                ls[j] = us[j] = v
    Lf, Uf = np.isfinite(ls), np.isfinite(us)
    fixc = Lf & Uf & (us - ls <= 0)
    Lf &= ~fixc
    Uf &= ~fixc
    rLf, rUf = np.isfinite(rls), np.isfinite(rus)
    eqr = rLf & rUf & (rus - rls <= 0) & (forced == 0)
    inq = (rLf | rUf) & ~eqr & (forced == 0)
    rLf &= inq
    rUf &= inq
    freer = ~(eqr | inq)
    cmask = (~fixc).astype(np.int32)
    rmask = (~freer).astype(np.int32)
    # K's values in the pattern's own CSR order (A may hold explicit zeros,
    # which scipy's products drop)
    rows = np.repeat(np.arange(m), np.diff(A.indptr))
    aval = dr[rows] * A.data * dc[A.indices]
    lp = np.where(Lf, ls, 0.0)
    up = np.where(Uf, us, 0.0)
    rlp = np.where(rLf, rls, 0.0)
    rup = np.where(rUf, rus, 0.0)
    beq = np.where(eqr, rls, 0.0)
    # ---- start point
    if x0 is None:
        x = np.clip(np.zeros(n), np.where(Lf, ls, -np.inf), np.where(Uf, us, np.inf))
        wid = np.where(Lf & Uf, us - ls, np.inf)
        th = np.minimum(push * np.maximum(1.0, np.abs(np.where(Lf, ls, np.where(Uf, us, 0.0)))), 0.5 * wid)
        x = np.where(Lf, np.maximum(x, ls + th), x)
        x = np.where(Uf, np.minimum(x, us - th), x)
        x = np.where(fixc, ls, x)
        ax = As @ x
        wr = np.where(rLf & rUf, rus - rls, np.inf)
        thr = np.minimum(push * np.maximum(1.0, np.abs(np.where(rLf, rls, np.where(rUf, rus, 0.0)))), 0.5 * wr)
        w = np.where(rLf, np.maximum(ax, rls + thr), ax)
        w = np.where(rUf, np.minimum(w, rus - thr), w)
        zl = np.where(Lf, 1.0, 0.0)
        zu = np.where(Uf, 1.0, 0.0)
        zlw = np.where(rLf, 1.0, 0.0)
        zuw = np.where(rUf, 1.0, 0.0)
        y = np.zeros(m)
        if zinit > 0:
            lam0 = gs + qs * x
            tl0 = np.where(Lf, x - np.where(Lf, ls, 0), 1.0)
            tu0 = np.where(Uf, np.where(Uf, us, 0) - x, 1.0)
            zl = np.where(Lf, np.maximum(lam0, 0) + zinit / tl0, 0.0)
            zu = np.where(Uf, np.maximum(-lam0, 0) + zinit / tu0, 0.0)
            # a one-sided column whose cost pushes towards its infinite side
            zl = np.where(Lf & ~Uf, np.maximum(zl, zinit), zl)
            zu = np.where(Uf & ~Lf, np.maximum(zu, zinit), zu)
            zlw = np.where(rLf, zinit / np.maximum(w - np.where(rLf, rls, 0), 1e-300), 0.0)
            zuw = np.where(rUf, zinit / np.maximum(np.where(rUf, rus, 0) - w, 1e-300), 0.0)
    else:
        x = x0 / dc
        y = y0 / dr / cs
        x = np.where(fixc, ls, x)
        mu = mu0
        wid = np.where(Lf & Uf, us - ls, np.inf)
        th = np.minimum(mu0 ** 0.5, 0.25 * wid)
        x = np.where(Lf, np.maximum(x, ls + th), x)
        x = np.where(Uf, np.minimum(x, us - th), x)
        ax = As @ x
        wr = np.where(rLf & rUf, rus - rls, np.inf)
        thr = np.minimum(mu0 ** 0.5, 0.25 * wr)
        w = np.where(rLf, np.maximum(ax, rls + thr), ax)
        w = np.where(rUf, np.minimum(w, rus - thr), w)
        lam = qs * x + gs - AsT @ y
        zl = np.where(Lf, np.maximum(lam, 0) + mu0 / np.maximum(x - lp, 1e-300), 0.0)
        zu = np.where(Uf, np.maximum(-lam, 0) + mu0 / np.maximum(up - x, 1e-300), 0.0)
        zlw = np.where(rLf, np.maximum(y, 0) + mu0 / np.maximum(w - rlp, 1e-300), 0.0)
        zuw = np.where(rUf, np.maximum(-y, 0) + mu0 / np.maximum(rup - w, 1e-300), 0.0)
    ncomp = Lf.sum() + Uf.sum() + rLf.sum() + rUf.sum()

    AT = sp.csr_matrix(A.T)

    def postsolve(xu, yu):
        # multipliers of the forced rows (unscaled): greedily the smallest
        # that gives every fixed column of the row the sign of its bound
        yu = yu.copy()
        yu[forced != 0] = 0.0
        lam = q * xu + g - AT @ yu
        for i in np.nonzero(forced)[0]:
            sl = slice(A.indptr[i], A.indptr[i + 1])
            cols, av = A.indices[sl], A.data[sl]
            nz = av != 0
            cols, av = cols[nz], av[nz]
            r = lam[cols] / av
            yi = max(0.0, np.max(r)) if forced[i] == 1 else min(0.0, np.min(r))
            if forced[i] == 1 and eqr_u[i]:
                yi = np.max(r)
            if forced[i] == -1 and eqr_u[i]:
                yi = np.min(r)
            yu[i] = yi
            lam[cols] -= av * yi
        return yu
    eqr_u = np.isfinite(rl) & np.isfinite(ru) & (ru - rl <= 0)
    lp_only = not np.any(qs > 0)
    hist = []
    t0 = time.time()
    for it in range(maxit):
        tl = np.where(Lf, x - lp, 1.0)
        tu = np.where(Uf, up - x, 1.0)
        tlw = np.where(rLf, w - rlp, 1.0)
        tuw = np.where(rUf, rup - w, 1.0)
        mu = (np.sum(tl * zl * Lf) + np.sum(tu * zu * Uf) + np.sum(tlw * zlw * rLf) + np.sum(tuw * zuw * rUf)) / ncomp
        # measure (unscaled)
        xu = x * dc
        yu = y * dr * cs
        ep, ed, eg, pobj, dobj = kkt_rel(xu, yu, g, q, A, rl, ru, l, u)
        hist.append((it, mu, ep, ed, eg))
        if verbose:
            print(f"  it {it:3d} mu {mu:.2e} ep {ep:.2e} ed {ed:.2e} eg {eg:.2e} pobj {pobj:.10e} dobj {dobj:.10e}")
        if forced.any():
            yu = postsolve(xu, yu)
            ep, ed, eg, pobj, dobj = kkt_rel(xu, yu, g, q, A, rl, ru, l, u)
            if verbose:
                print(f"      postsolved: ep {ep:.2e} ed {ed:.2e} eg {eg:.2e} dobj {dobj:.10e}")
        if ep <= tol and ed <= tol and eg <= tol:
            return xu, yu, 0, it, hist
        ax = As @ x
        rpx = np.where(eqr, beq - ax, np.where(inq, w - ax, 0.0))   # primal: A dx - dw = rp
        rdx = qs * x + gs - AsT @ y - zl + zu
        rdx = np.where(fixc, 0.0, rdx)
        rdw = np.where(inq, y - zlw + zuw, 0.0)
        Sx = np.where(Lf, zl / tl, 0.0) + np.where(Uf, zu / tu, 0.0)
        Sw = np.where(rLf, zlw / tlw, 0.0) + np.where(rUf, zuw / tuw, 0.0)
        Hd = qs + Sx + delta
        Hd = np.where(fixc, 1.0, Hd)
        Gi = np.where(inq, 1.0 / np.maximum(Sw, 1e-300), 0.0)
        Gd = -(Gi + delta)
        Gd = np.where(freer, -1.0, Gd)
        diag = np.concatenate([Hd, Gd])
        F.factor(diag, aval, cmask, rmask, delta)
        Hx = qs + Sx  # the unregularised system for refinement
        Hx = np.where(fixc, 1.0, Hx)

        def kmul(dx, dy):
            ox = Hx * dx - np.where(fixc, 0, AsT @ np.where(freer, 0, dy))
            oy = -(As @ np.where(fixc, 0, dx)) - Gi * dy
            oy = np.where(freer, -dy, oy)
            return ox, oy

        def ksolve(bx, by):
            z = F.solve(np.concatenate([bx, by]))
            dx, dy = z[:n], z[n:]
            for _ in range(refine):
                ox, oy = kmul(dx, dy)
                rx, ry = bx - ox, by - oy
                if max(np.max(np.abs(rx)), np.max(np.abs(ry))) <= 1e-14 * max(1.0, np.max(np.abs(bx)), np.max(np.abs(by))):
                    break
                z = F.solve(np.concatenate([rx, ry]))
                dx, dy = dx + z[:n], dy + z[n:]
            return dx, dy

        def direction(rcl, rcu, rclw, rcuw):
            # H dx - A'dy = -rdx + rcl/tl - rcu/tu ; row: -(A dx + Gi dy) = -(rp + (xi_w)/Sw)
            bx = -rdx + np.where(Lf, rcl / tl, 0) - np.where(Uf, rcu / tu, 0)
            bx = np.where(fixc, 0.0, bx)
            xiw = -rdw + np.where(rLf, rclw / tlw, 0) - np.where(rUf, rcuw / tuw, 0)
            by = -(rpx + Gi * xiw)
            by = np.where(freer, 0.0, by)
            dx, dy = ksolve(bx, by)
            dw = np.where(inq, As @ dx - rpx, 0.0)
            dzl = np.where(Lf, (rcl - zl * dx) / tl, 0)
            dzu = np.where(Uf, (rcu + zu * dx) / tu, 0)
            dzlw = np.where(rLf, (rclw - zlw * dw) / tlw, 0)
            dzuw = np.where(rUf, (rcuw + zuw * dw) / tuw, 0)
            return dx, dy, dw, dzl, dzu, dzlw, dzuw

        def steps(dx, dw, dzl, dzu, dzlw, dzuw):
            def mx(t, d, mask):
                r = np.where(mask & (d < 0), -t / np.where(d < 0, d, -1), np.inf)
                return np.min(r, initial=np.inf)
            ap = min(mx(tl, dx, Lf), mx(tu, -dx, Uf), mx(tlw, dw, rLf), mx(tuw, -dw, rUf))
            ad = min(mx(zl, dzl, Lf), mx(zu, dzu, Uf), mx(zlw, dzlw, rLf), mx(zuw, dzuw, rUf))
            return ap, ad

        # predictor
        dxa, dya, dwa, dzla, dzua, dzlwa, dzuwa = direction(-tl * zl, -tu * zu, -tlw * zlw, -tuw * zuw)
        apa, ada = steps(dxa, dwa, dzla, dzua, dzlwa, dzuwa)
        apa, ada = min(1.0, apa), min(1.0, ada)
        if not lp_only:
            apa = ada = min(apa, ada)
        mua = (np.sum(((tl + apa * dxa) * (zl + ada * dzla))[Lf]) + np.sum(((tu - apa * dxa) * (zu + ada * dzua))[Uf])
               + np.sum(((tlw + apa * dwa) * (zlw + ada * dzlwa))[rLf])
               + np.sum(((tuw - apa * dwa) * (zuw + ada * dzuwa))[rUf])) / ncomp
        sig = min(sigmax, (mua / mu) ** 3)
        sm = sig * mu
        dx, dy, dw, dzl, dzu, dzlw, dzuw = direction(sm - tl * zl - dxa * dzla, sm - tu * zu + dxa * dzua,
                                                     sm - tlw * zlw - dwa * dzlwa, sm - tuw * zuw + dwa * dzuwa)
        ap, ad = steps(dx, dw, dzl, dzu, dzlw, dzuw)
        if center_fb > 0 and min(ap, ad) < center_fb:
            # a blocked step: a pure centring direction instead (sigma 0.9)
            sm = 0.9 * mu
            dx, dy, dw, dzl, dzu, dzlw, dzuw = direction(sm - tl * zl, sm - tu * zu, sm - tlw * zlw, sm - tuw * zuw)
            ap, ad = steps(dx, dw, dzl, dzu, dzlw, dzuw)
        eta = max(0.9, 1.0 - 10 * mu) if True else 0.99
        eta = min(eta, eta_max)
        ap, ad = min(1.0, eta * ap), min(1.0, eta * ad)
        if not lp_only or same_step:
            ap = ad = min(ap, ad)
        x = x + ap * dx
        w = w + ap * dw
        y = y + ad * dy
        zl = zl + ad * dzl
        zu = zu + ad * dzu
        zlw = zlw + ad * dzlw
        zuw = zuw + ad * dzuw
    return x * dc, y * dr * cs, 1, maxit, hist


def uc_case(S):
    from mpisppy_amd.examples import uc
    names = uc.all_scenario_names(S)
    return uc.batch_creator(names)


if __name__ == "__main__":
    kind = sys.argv[1] if len(sys.argv) > 1 else "uc"
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    d = uc_case(S)
    n, m = d.n, d.m
    F = Factor(n, m, d.row_ptr, d.col_idx)
    print("factor info N ns nlev panel u flops nnzL:", F.info[:7].tolist())
    A = sp.csr_matrix((d.vals[:, 0], d.col_idx, d.row_ptr), shape=(m, n))
    dr, dc = ruiz_pc(A)
    import json
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "uc_lp_values.json")))
    for s in range(S):
        t = time.time()
        kw = eval('dict(' + (sys.argv[3] if len(sys.argv) > 3 else '') + ')')
        x, y, st, it, hist = ipm(F, A, d.c[:, s], np.zeros(n), d.l[:, s], d.u[:, s], d.rl[:, s], d.ru[:, s], dr, dc,
                                 verbose=True, **kw)
        ep, ed, eg, pobj, dobj = kkt_rel(x, y, d.c[:, s], np.zeros(n), A, d.rl[:, s], d.ru[:, s], d.l[:, s], d.u[:, s])
        nm = d.names[s]
        print(f"{nm}: status {st} its {it} pobj {pobj + d.const[s]:.10f} gold {gold['values'].get(nm)} "
              f"dobj {dobj + d.const[s]:.10f} ({time.time() - t:.1f}s)")


def polish(F, A, g, q, l, u, rl, ru, x, y, dr, dc, delta=1e-9, refine=20, rounds=4, verbose=True):
    """Active-set polish of an (approximate) optimum on the ORIGINAL problem:
    classify by the primal-dual active-set rule, solve the active set's
    regularised KKT system (refined against the unregularised one), check."""
    n, m = A.shape[1], A.shape[0]
    rows = np.repeat(np.arange(m), np.diff(A.indptr))
    As = sp.csr_matrix((dr[rows] * A.data * dc[A.indices], A.indices, A.indptr), shape=(m, n))
    AsT = sp.csr_matrix(As.T)
    aval = As.data
    gs, qs = g * dc, q * dc * dc
    ls, us, rls, rus = l / dc, u / dc, rl * dr, ru * dr
    xs, ys = x / dc, y / dr
    for rd in range(rounds):
        lam = qs * xs + gs - AsT @ ys
        ax = As @ xs
        atl = np.isfinite(ls) & (lam + (ls - xs) > 0)
        atu = np.isfinite(us) & (lam + (us - xs) < 0) & ~atl
        fixed = atl | atu | (ls == us)
        xb = np.where(atl, ls, np.where(atu, us, np.where(ls == us, ls, 0.0)))
        rat_l = np.isfinite(rls) & (ys + (rls - ax) > 0)
        rat_u = np.isfinite(rus) & (ys + (rus - ax) < 0) & ~rat_l
        act = rat_l | rat_u
        b = np.where(rat_l, rls, np.where(rat_u, rus, 0.0))
        cm = (~fixed).astype(np.int32)
        rm = act.astype(np.int32)
        Hd = np.where(fixed, 1.0, qs + delta)
        Gd = np.where(act, -delta, -1.0)
        F.factor(np.concatenate([Hd, Gd]), aval, cm, rm, delta)
        # unknowns: x_F, y_R (fixed x = bound, inactive y = 0)
        Afx = As @ np.where(fixed, xb, 0.0)
        bx = np.where(fixed, 0.0, -gs)
        by = np.where(act, -(b - Afx), 0.0)
        H0 = np.where(fixed, 1.0, qs)

        def kmul(dxv, dyv):
            ox = H0 * dxv - np.where(fixed, 0, AsT @ np.where(act, dyv, 0))
            oy = np.where(act, -(As @ np.where(fixed, 0, dxv)), -dyv)
            return ox, oy
        z = F.solve(np.concatenate([bx, by]))
        dxv, dyv = z[:n], z[n:]
        for _ in range(refine):
            ox, oy = kmul(dxv, dyv)
            rx, ry = bx - ox, by - oy
            if max(np.abs(rx).max(), np.abs(ry).max()) <= 1e-15 * max(1, np.abs(bx).max(), np.abs(by).max()):
                break
            z = F.solve(np.concatenate([rx, ry]))
            dxv, dyv = dxv + z[:n], dyv + z[n:]
        xs = np.where(fixed, xb, np.clip(dxv, ls, us))
        ys = np.where(act, dyv, 0.0)
        ep, ed, eg, pobj, dobj = kkt_rel(xs * dc, ys * dr, g, q, A, rl, ru, l, u)
        if verbose:
            ox, oy = kmul(dxv, dyv)
            print(f"   polish round {rd}: fixed {fixed.sum()} active rows {act.sum()} ep {ep:.2e} ed {ed:.2e} "
                  f"eg {eg:.2e} pobj {pobj:.10f} res {np.abs(bx-ox).max():.1e} {np.abs(by-oy).max():.1e} "
                  f"clip {np.abs(np.clip(dxv, ls, us) - dxv).max():.1e}")
        if ep <= 1e-9 and ed <= 1e-9 and eg <= 1e-9:
            return xs * dc, ys * dr, 0
    return xs * dc, ys * dr, 1


def polish_prox(F, A, g, q, l, u, rl, ru, x, y, dr, dc, delta=1e-9, inner=8, rounds=3, verbose=True):
    """Active-set polish as proximal-point corrections from the given point:
    the active set's equations (free columns: reduced cost 0; active rows:
    at their bound) solved by steps of K_delta [dx; dy] = -residual, which
    move the iterate only in the range of the active set's equations (the
    null directions of a degenerate LP stay where the interior point put
    them)."""
    n, m = A.shape[1], A.shape[0]
    rows = np.repeat(np.arange(m), np.diff(A.indptr))
    As = sp.csr_matrix((dr[rows] * A.data * dc[A.indices], A.indices, A.indptr), shape=(m, n))
    AsT = sp.csr_matrix(As.T)
    aval = As.data
    gs, qs = g * dc, q * dc * dc
    ls, us, rls, rus = l / dc, u / dc, rl * dr, ru * dr
    xs, ys = x / dc, y / dr
    best = None
    for rd in range(rounds):
        lam = qs * xs + gs - AsT @ ys
        ax = As @ xs
        # classify: complementarity split (the interior point's t vs z)
        atl = np.isfinite(ls) & (lam + (ls - xs) > 0)
        atu = np.isfinite(us) & (lam + (us - xs) < 0) & ~atl
        fixed = atl | atu | (ls == us)
        xb = np.where(atl, ls, np.where(atu, us, np.where(ls == us, ls, 0.0)))
        rat_l = np.isfinite(rls) & (ys + (rls - ax) > 0)
        rat_u = np.isfinite(rus) & (ys + (rus - ax) < 0) & ~rat_l
        act = rat_l | rat_u
        b = np.where(rat_l, rls, np.where(rat_u, rus, 0.0))
        cm = (~fixed).astype(np.int32)
        rm = act.astype(np.int32)
        Hd = np.where(fixed, 1.0, qs + delta)
        Gd = np.where(act, -delta, -1.0)
        F.factor(np.concatenate([Hd, Gd]), aval, cm, rm, delta)
        xs = np.where(fixed, xb, xs)
        ys = np.where(act, ys, 0.0)
        for it in range(inner):
            lam = qs * xs + gs - AsT @ ys
            rdv = np.where(fixed, 0.0, lam)
            rpv = np.where(act, b - As @ xs, 0.0)
            z = F.solve(np.concatenate([-rdv, -rpv]))
            xs = np.where(fixed, xs, xs + z[:n])
            ys = np.where(act, ys + z[n:], 0.0)
            xc = np.clip(xs, ls, us)
            ep, ed, eg, pobj, dobj = kkt_rel(xc * dc, ys * dr, g, q, A, rl, ru, l, u)
            if verbose:
                print(f"   prox polish round {rd} it {it}: fixed {fixed.sum()} active {act.sum()} ep {ep:.2e} ed {ed:.2e} "
                      f"eg {eg:.2e} pobj {pobj:.10f} |rd| {np.abs(rdv).max():.1e} |rp| {np.abs(rpv).max():.1e} "
                      f"clip {np.abs(xc - xs).max():.1e}")
            if ep <= 1e-9 and ed <= 1e-9 and eg <= 1e-9:
                return xc * dc, ys * dr, 0
        xs = np.clip(xs, ls, us)
    return xs * dc, ys * dr, 1
