"""Oracle restatement of the reference PH control flow (TEST INFRASTRUCTURE).

Follows ``mpisppy/phbase.py`` and ``mpisppy/opt/ph.py`` line by line in
semantics (not in code), single process, emulating the reference's
``n_proc``-rank scenario slicing where the result depends on it
(``convergence_diff``, ``phbase.py:254-276``).
"""
import math
import numpy as np

from .solve import solve_scenario


def rank_slices(num_scens, n_proc):
    """``mpisppy/utils/sputils.py:619-628`` (``_ScenTree.scen_names_to_ranks``)."""
    if n_proc == 1:
        return [list(range(num_scens))]
    avg = num_scens / n_proc
    return [list(range(int(i * avg), int((i + 1) * avg))) for i in range(n_proc)]


class OraclePH:
    """PH over a list of :class:`oracle.models.OScen` (all scenarios, in order)."""

    def __init__(self, options, scens, n_proc=1, variable_prob=None, bundles=None):
        self.options = dict(options)
        # bundles: lists of scenario indices solved as one EF subproblem
        # (spbase.py:206-240, phbase.py:803-862 / 1273-1302); None: each
        # scenario is a subproblem
        self.bundles = None if bundles is None else [list(b) for b in bundles]
        self.scens = scens
        self.S = len(scens)
        self.n_proc = n_proc
        self.slices = rank_slices(self.S, n_proc)
        # spbase.py:486-490 -- uniform probability when not attached
        self.prob = np.array([s.prob if s.prob is not None else 1.0 / self.S for s in scens])
        self.is_min = scens[0].sense == "min"
        # spbase.py:353-366 -- prob_coeff[node] = p_s / uncond_prob(node)
        self.prob_coeff = []
        for s, p in zip(scens, self.prob):
            unc = 1.0
            pcs = []
            for i, (nm, cp, idx) in enumerate(s.nodes):
                unc = unc * cp if i > 0 else 1.0
                pcs.append(p / unc)
            self.prob_coeff.append(pcs)
        rho0 = float(self.options["defaultPHrho"])
        self.K = [len(s.nonant_idx) for s in scens]
        # per nonant slot weights; variable probabilities (spbase.py:369-400)
        # replace a slot's prob_coeff and mask its W when zero (phbase.py:246-251)
        self.pc_slot = []
        self.w_coeff = []
        for s, sc in enumerate(scens):
            pcs = np.concatenate([np.full(len(idx), self.prob_coeff[s][j])
                                  for j, (nm, cp, idx) in enumerate(sc.nodes)])
            wc = np.ones(len(pcs))
            for k, p in (variable_prob or {}).get(s, {}).items():
                pcs[k] = p
                if p == 0:
                    wc[k] = 0.0
            self.pc_slot.append(pcs)
            self.w_coeff.append(wc)
        self.W = [np.zeros(k) for k in self.K]           # phbase.py:1113-1115
        self.rho = [np.full(k, rho0) for k in self.K]    # phbase.py:1128-1131
        self.xbar = [np.zeros(k) for k in self.K]        # phbase.py:1622-1632
        self.xsqbar = [np.zeros(k) for k in self.K]
        self.w_on = 0.0                                  # attached disabled
        self.prox_on = 0.0
        self.x = [None] * self.S
        self.outer_bound = np.zeros(self.S)
        self.feasible = np.ones(self.S, dtype=bool)
        self.solve_count = 0
        self.conv = None
        self.history = {"conv": [], "xbar": []}

    # -------------------------------------------------------------- model --
    def _cmin(self, s):
        sc = self.scens[s]
        return sc.c if self.is_min else -sc.c

    def _terms(self, s, w_on, prox_on):
        """Min-form (g, q, const) of the PH-augmented objective (phbase.py:1133-1209)."""
        sc = self.scens[s]
        idx = sc.nonant_idx
        g = self._cmin(s).copy()
        q = np.zeros_like(g)
        const = sc.const if self.is_min else -sc.const
        np.add.at(g, idx, w_on * self.W[s] - prox_on * self.rho[s] * self.xbar[s])
        np.add.at(q, idx, prox_on * self.rho[s])
        const += prox_on * float(np.sum(self.rho[s] / 2.0 * self.xbar[s] ** 2))
        return g, q, const

    def objective(self, s, x=None, w_on=None, prox_on=None):
        """Value of the scenario's *active objective* in the reference's sense."""
        x = self.x[s] if x is None else x
        w_on = self.w_on if w_on is None else w_on
        prox_on = self.prox_on if prox_on is None else prox_on
        g, q, const = self._terms(s, w_on, prox_on)
        v = 0.5 * float(np.dot(q * x, x)) + float(np.dot(g, x)) + const
        return v if self.is_min else -v

    # -------------------------------------------------------------- solve --
    def _solve_bundle(self, b, members, w_on, prox_on):
        """One bundle: the EF of its scenarios (sputils.py:246-383) -- the
        PH-augmented scenario objectives weighted by p_s and normalised by the
        bundle probability P_b, nonanticipativity rows x_s[k] == x_ref[k]
        per tree node (ref: the bundle's first scenario at the node) -- solved
        exactly; every member gets its block of the solution, the bundle its
        outer bound (phbase.py:985-995)."""
        import scipy.sparse as sp
        P = float(sum(self.prob[s] for s in members))
        gs, qs, cst = [], [], 0.0
        for s in members:
            g, q, c0 = self._terms(s, w_on, prox_on)
            wt = self.prob[s] / P
            gs.append(wt * g)
            qs.append(wt * q)
            cst += wt * c0
        ns = [self.scens[s].A.shape[1] for s in members]
        offs = np.concatenate([[0], np.cumsum(ns)]).astype(int)
        A = sp.block_diag([self.scens[s].A for s in members], format="csr")
        rl = [np.concatenate([self.scens[s].rl for s in members])]
        ru = [np.concatenate([self.scens[s].ru for s in members])]
        first = {}
        link = []
        for t, s in enumerate(members):
            for (nm, cp, idx) in self.scens[s].nodes:
                if nm not in first:
                    first[nm] = (t, idx)
                    continue
                t0, idx0 = first[nm]
                for a, r in zip(idx, idx0):
                    link.append((offs[t] + a, offs[t0] + r))
        if link:
            na = sp.csr_matrix((np.tile([1.0, -1.0], len(link)),
                                (np.repeat(np.arange(len(link)), 2), np.array(link).reshape(-1))),
                               shape=(len(link), offs[-1]))
            A = sp.vstack([A, na]).tocsr()
            rl.append(np.zeros(len(link)))
            ru.append(np.zeros(len(link)))
        g, q = np.concatenate(gs), np.concatenate(qs)
        l = np.concatenate([self.scens[s].l for s in members])
        u = np.concatenate([self.scens[s].u for s in members])
        x, y, feas = solve_scenario(g, q, A, np.concatenate(rl), np.concatenate(ru), l, u)
        for t, s in enumerate(members):
            self.feasible[s] = feas
            if feas:
                self.x[s] = x[offs[t]:offs[t + 1]].copy()
        if feas:
            v = 0.5 * float(np.dot(q * x, x)) + float(np.dot(g, x)) + cst
            self.bundle_bound[b] = v if self.is_min else -v
        self.solve_count += 1

    def solve_loop(self, w_on=None, prox_on=None):
        """phbase.py:999-1095 + solve_one 864-996."""
        w_on = self.w_on if w_on is None else w_on
        prox_on = self.prox_on if prox_on is None else prox_on
        if self.bundles is not None:
            if not hasattr(self, "bundle_bound"):
                self.bundle_bound = np.zeros(len(self.bundles))
            for b, members in enumerate(self.bundles):
                self._solve_bundle(b, members, w_on, prox_on)
            return
        for s in range(self.S):
            sc = self.scens[s]
            g, q, const = self._terms(s, w_on, prox_on)
            x, y, feas = solve_scenario(g, q, sc.A, sc.rl, sc.ru, sc.l, sc.u)
            self.feasible[s] = feas
            if feas:
                self.x[s] = x
                v = 0.5 * float(np.dot(q * x, x)) + float(np.dot(g, x)) + const
                # exact solve: Lower_bound == optimum (phbase.py:985-988)
                self.outer_bound[s] = v if self.is_min else -v
            self.solve_count += 1

    # ---------------------------------------------------------- PH pieces --
    def _node_groups(self):
        groups = {}
        for s, sc in enumerate(self.scens):
            off = 0
            for j, (nm, cp, idx) in enumerate(sc.nodes):
                groups.setdefault(nm, []).append((s, off, len(idx), j))
                off += len(idx)
        return groups

    def Compute_Xbar(self):
        """phbase.py:144-221."""
        for nm, members in self._node_groups().items():
            nlen = members[0][2]
            acc = np.zeros(nlen)
            accsq = np.zeros(nlen)
            for (s, off, ln, j) in members:
                xs = self.x[s][self.scens[s].nonant_idx[off:off + ln]]
                pc = self.pc_slot[s][off:off + ln]
                acc += pc * xs
                accsq += pc * xs ** 2
            for (s, off, ln, j) in members:
                self.xbar[s][off:off + ln] = acc
                self.xsqbar[s][off:off + ln] = accsq

    def Update_W(self):
        """phbase.py:224-251 (W masked by w_coeff after the update)."""
        for s in range(self.S):
            xs = self.x[s][self.scens[s].nonant_idx]
            self.W[s] = (self.W[s] + self.rho[s] * (xs - self.xbar[s])) * self.w_coeff[s]

    def convergence_diff(self):
        """phbase.py:254-276: sum over ranks of local mean |x-xbar|, / n_proc."""
        tot = 0.0
        for sl in self.slices:
            d = 0.0
            cnt = 0
            for s in sl:
                xs = self.x[s][self.scens[s].nonant_idx]
                d += float(np.sum(np.abs(xs - self.xbar[s])))
                cnt += xs.size
            tot += d / cnt
        return tot / self.n_proc

    def Eobjective(self):
        """phbase.py:279-312."""
        return math.fsum(self.prob[s] * self.objective(s) for s in range(self.S))

    def Ebound(self):
        """phbase.py:314-354 (over subproblems: a bundle weighs P_b)."""
        if self.bundles is not None:
            return math.fsum(float(sum(self.prob[s] for s in mem)) * self.bundle_bound[b]
                             for b, mem in enumerate(self.bundles))
        return math.fsum(self.prob[s] * self.outer_bound[s] for s in range(self.S))

    # ------------------------------------------------------------ drivers --
    def Iter0(self):
        """phbase.py:1364-1470 (W and prox attached but disabled)."""
        self.solve_loop(0.0, 0.0)
        if not np.all(self.feasible):
            raise RuntimeError("Infeasibility detected in Iter0")
        self.trivial_bound = self.Ebound()
        self.w_on = 1.0
        self.prox_on = 1.0
        return self.trivial_bound

    def iterk_loop(self):
        """phbase.py:1472-1566 (no extensions / converger / spcomm)."""
        self.conv = None
        maxit = int(self.options["PHIterLimit"])
        self.iters = 0
        for it in range(1, maxit + 1):
            self.iters = it
            self.Compute_Xbar()
            self.Update_W()
            self.conv = self.convergence_diff()
            self.history["conv"].append(self.conv)
            self.history["xbar"].append([xb.copy() for xb in self.xbar])
            if self.conv < self.options["convthresh"]:
                break
            self.solve_loop()

    def ph_main(self):
        """opt/ph.py:26-72 -> (conv, Eobj, trivial_bound)."""
        tb = self.Iter0()
        self.iterk_loop()
        eobj = self.Eobjective()
        return self.conv, eobj, tb

    def post_solve_bound(self):
        """phbase.py:753-801: W on, prox off, LP solves, Ebound."""
        self.solve_loop(1.0, 0.0)
        return self.Ebound()

    def lagrangian_bound(self, W=None):
        """cylinders/lagrangian_bounder.py:19-57 -- solve_loop (W, no prox) + Ebound."""
        if W is not None:
            self.W = [np.array(w, dtype=np.float64) for w in W]
        self.solve_loop(1.0, 0.0)
        return self.Ebound()


def xhat_objective(scens, xhat_by_node, prob=None):
    """extensions/xhatbase.py:_try_one restated: every scenario's nonants at
    node nd fixed at xhat_by_node[nd] (in the node's nonant order), the
    scenario LPs solved exactly (W and prox off), the expected objective in
    the reference's sense; None if a scenario is infeasible."""
    S = len(scens)
    prob = np.array([s.prob if s.prob is not None else 1.0 / S for s in scens]) if prob is None \
        else np.asarray(prob)
    tot = []
    for p, sc in zip(prob, scens):
        l, u = sc.l.copy(), sc.u.copy()
        for (nm, cp, idx) in sc.nodes:
            v = np.asarray(xhat_by_node[nm], dtype=np.float64)
            l[idx] = v
            u[idx] = v
        sgn = 1.0 if sc.sense == "min" else -1.0
        x, y, feas = solve_scenario(sgn * sc.c, None, sc.A, sc.rl, sc.ru, l, u)
        if not feas:
            return None
        tot.append(p * (float(sc.c @ x) + sc.const))
    return math.fsum(tot)
