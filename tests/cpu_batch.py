"""Test-only stand-in for DeviceBatch on CPU tensors.

Implements the device operations PHBase calls (solve, summary, xbar_accum,
update_w, segment_sum, eval_objective) with torch CPU ops and the oracle's
exact per-scenario solver, so the distributed *host* logic of PHBase
(slicing, node slots, allreduces, convergence bookkeeping) can be tested
with gloo on a machine without a GPU.  Never used by the product.
"""
import numpy as np
import scipy.sparse as sp
import torch

from oracle.solve import solve_scenario


class CPUBatch:
    def __init__(self, data):
        self.data = data
        self.S, self.n, self.m, self.nnz, self.K = data.S, data.n, data.m, data.nnz, data.K
        f64 = dict(dtype=torch.float64)
        self.x = torch.zeros(self.n * self.S, **f64)
        self.y = torch.zeros(max(self.m, 1) * self.S, **f64)
        self.status = torch.zeros(self.S, dtype=torch.int32)
        self.iters = torch.zeros(self.S, dtype=torch.int32)
        self.pobj = torch.zeros(self.S, **f64)
        self.dbound = torch.zeros(self.S, **f64)
        self.const = torch.as_tensor(data.const, **f64)
        self.cols = torch.as_tensor(data.nonant_cols.astype(np.int64))

    def _A(self, s):
        d = self.data
        return sp.csr_matrix((d.vals[:, s], d.col_idx, d.row_ptr), shape=(d.m, d.n))

    # ---- device-loop emulation (ph_loop_* semantics of include/phgpu.h)
    _loop = False
    _ctl = None

    _xa = None

    def loop_reset(self, start_iter, iter_limit, convthresh):
        self._ctl = dict(stop=0, iter=int(start_iter), limit=int(iter_limit),
                         thresh=float(convthresh), acc=[0, 0, 0, 0, 0, 0])
        self._advance()

    def _advance(self):
        c = self._ctl
        if c["stop"]:
            return
        if c["iter"] >= c["limit"]:
            c["stop"] = 2
        else:
            c["iter"] += 1

    def loop_enable(self, on):
        self._loop = bool(on)

    def _stopped(self):
        return self._loop and self._ctl["stop"] != 0

    def loop_set_xbar(self, prob_coeff, slot_k, slot_s0, slot_s1, out):
        self._xa = None if slot_k is None else (prob_coeff, slot_k, slot_s0, slot_s1, out)

    def loop_conv_local(self, absdiff, seg, cnt, nproc, parts, conv_hist):
        if self._stopped():
            return
        self.segment_sum(absdiff, None, seg, parts)
        self.loop_conv(parts, cnt, nproc, conv_hist)

    def loop_update_w_conv(self, sums, G, gid, rho, w_coeff, xbar, xsqbar, W, absdiff, wconv,
                           conv_hist):
        if self._stopped():
            return
        self.update_w(sums, G, gid, rho, w_coeff, xbar, xsqbar, W, absdiff)
        c = self._ctl
        v = float((absdiff * wconv).sum())
        conv_hist[c["iter"] - 1] = v
        if v < c["thresh"]:
            c["stop"] = 1

    def loop_conv(self, parts, cnt, nproc, conv_hist):
        c = self._ctl
        if c["stop"]:
            return
        v = 0.0
        for r in range(parts.numel()):
            v += float(parts[r]) / float(cnt[r])
        v /= nproc
        conv_hist[c["iter"] - 1] = v
        if v < c["thresh"]:
            c["stop"] = 1

    def loop_conv_lagged(self, parts, cnt, nproc, conv_hist):
        c = self._ctl
        if c["stop"] == 1:
            return
        k = c.get("pend", 0)
        if k > 0:
            v = 0.0
            for r in range(parts.numel()):
                v += float(parts[r]) / (float(cnt[r]) if cnt is not None else 1.0)
            v /= nproc
            conv_hist[k - 1] = v
            c["pend"] = 0
            if v < c["thresh"]:
                c["stop"] = 1
                c["iter"] = k

    def loop_backup(self, x_save, y_save):
        if self._stopped():
            return
        x_save.copy_(self.x)
        y_save.copy_(self.y)
        self._ctl["pend"] = self._ctl["iter"]

    def loop_backup_status(self, status_save, dbound_save):
        if self._stopped():
            return
        status_save.copy_(self.status)
        dbound_save.copy_(self.dbound)

    _pass = None

    def loop_bind_pass(self, sums, G, gid, rho, w_coeff, xbar, xsqbar, W, absdiff, wconv,
                       conv_hist, conv_part, saves, w_on, prox_on, **kw):
        self._pass = dict(sums=sums, G=G, gid=gid, rho=rho, w_coeff=w_coeff, xbar=xbar,
                          xsqbar=xsqbar, W=W, absdiff=absdiff, wconv=wconv, conv_hist=conv_hist,
                          conv_part=conv_part, saves=saves, w_on=w_on, prox_on=prox_on)

    def loop_unbind_pass(self):
        self._pass = None

    def loop_pass(self):
        """ph_loop_pass semantics (include/phgpu.h)."""
        p = self._pass
        if p["conv_part"] is None:
            self.loop_update_w_conv(p["sums"], p["G"], p["gid"], p["rho"], p["w_coeff"],
                                    p["xbar"], p["xsqbar"], p["W"], p["absdiff"], p["wconv"],
                                    p["conv_hist"])
        else:
            self.loop_conv_lagged(p["conv_part"], None, 1.0, p["conv_hist"])
            if not self._stopped():
                self.update_w(p["sums"], p["G"], p["gid"], p["rho"], p["w_coeff"], p["xbar"],
                              p["xsqbar"], p["W"], p["absdiff"])
                p["conv_part"][0] = float((p["absdiff"] * p["wconv"]).sum())
                xs, ys, ss, ds = p["saves"]
                self.loop_backup(xs, ys)
                self.loop_backup_status(ss, ds)
        self.solve(p["W"], p["rho"], p["xbar"], p["w_on"], p["prox_on"])

    def loop_run(self, iters):
        """ph_loop_run semantics: up to `iters` passes (the stop flag ends it)."""
        for _ in range(int(iters)):
            if self._stopped():
                break
            self.loop_pass()

    def loop_status(self):
        c = self._ctl
        return (c["stop"], c["iter"], *c["acc"])

    def solve(self, W, rho, xbar, w_on, prox_on, **kw):
        if self._stopped():
            return
        self._solve(W, rho, xbar, w_on, prox_on)
        if self._loop:
            a = self._ctl["acc"]
            a[0] += int(np.sum(self.status.numpy() != 0))
            a[1] += self.S
            if self._xa is not None:
                self.xbar_accum(*self._xa)
            self._advance()

    _lu = None

    def set_bounds(self, l, u):
        self._lu = (l.view(self.n, self.S).numpy().copy(), u.view(self.n, self.S).numpy().copy())

    @property
    def l(self):
        return torch.as_tensor(self.data.l.reshape(-1).copy())

    @property
    def u(self):
        return torch.as_tensor(self.data.u.reshape(-1).copy())

    def _solve(self, W, rho, xbar, w_on, prox_on):
        d = self.data
        L, U = (d.l, d.u) if self._lu is None else self._lu
        Wv = W.view(self.K, self.S).numpy(); rv = rho.view(self.K, self.S).numpy()
        xb = xbar.view(self.K, self.S).numpy()
        X = self.x.view(self.n, self.S)
        for s in range(self.S):
            g = d.c[:, s].copy(); q = np.zeros(self.n)
            g[d.nonant_cols] += w_on * Wv[:, s] - prox_on * rv[:, s] * xb[:, s]
            q[d.nonant_cols] += prox_on * rv[:, s]
            cst = prox_on * float(np.sum(rv[:, s] / 2 * xb[:, s] ** 2))
            x, y, feas = solve_scenario(g, q, self._A(s), d.rl[:, s], d.ru[:, s], L[:, s], U[:, s])
            X[:, s] = torch.as_tensor(x)
            v = 0.5 * float(q @ (x * x)) + float(g @ x) + cst
            self.pobj[s] = v
            self.dbound[s] = v
            self.status[s] = 0

    def summary(self):
        st = self.status.numpy()
        it = self.iters.numpy()
        return int(np.sum(st != 0)), int(it.sum()), int(it.max(initial=0)), 0, 0

    def xbar_accum(self, prob_coeff, slot_k, slot_s0, slot_s1, out):
        if self._stopped():
            return
        X = self.x.view(self.n, self.S)[self.cols]
        pc = prob_coeff.view(self.K, self.S)
        G = slot_k.numel()
        for g in range(G):
            k, a, b = int(slot_k[g]), int(slot_s0[g]), int(slot_s1[g])
            out[g] = (pc[k, a:b] * X[k, a:b]).sum()
            out[G + g] = (pc[k, a:b] * X[k, a:b] ** 2).sum()

    def update_w(self, sums, G, gid, rho, w_coeff, xbar, xsqbar, W, absdiff):
        if self._stopped():
            return
        X = self.x.view(self.n, self.S)[self.cols]
        gi = gid.view(self.K, self.S).long()
        xb = sums[:G][gi]
        xbar.view(self.K, self.S).copy_(xb)
        xsqbar.view(self.K, self.S).copy_(sums[G:][gi])
        d = X - xb
        if W is not None:
            Wv = W.view(self.K, self.S)
            Wv.add_(rho.view(self.K, self.S) * d)
            if w_coeff is not None:
                Wv.mul_(w_coeff.view(self.K, self.S))
        absdiff.copy_(d.abs().sum(0))

    def segment_sum(self, v, w, seg, out):
        if self._stopped():
            return
        for r in range(seg.numel() - 1):
            a, b = int(seg[r]), int(seg[r + 1])
            out[r] = (v[a:b] * (w[a:b] if w is not None else 1.0)).sum()

    def gather(self, src, idx, wt, count, dst):
        i = idx.long()
        v = torch.where(i >= 0, src[i.clamp(min=0)], torch.zeros_like(dst))
        dst.copy_(v * wt if wt is not None else v)

    def eval_objective(self, W, rho, xbar, w_on, prox_on, out):
        d = self.data
        X = self.x.view(self.n, self.S)
        out.copy_((torch.as_tensor(d.c) * X).sum(0))
        Xn = X[self.cols]
        Wv = W.view(self.K, self.S); rv = rho.view(self.K, self.S); xb = xbar.view(self.K, self.S)
        out.add_((w_on * Wv * Xn + prox_on * 0.5 * rv * (Xn ** 2 - 2 * xb * Xn + xb ** 2)).sum(0))
