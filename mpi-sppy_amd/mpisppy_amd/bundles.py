"""Bundles (``PHoptions["bundles_per_rank"]``): several scenarios solved as
ONE subproblem, their extensive form.

Reference: ``spbase.py:206-240`` (``_assign_bundles``: contiguous slices of
each rank's scenarios), ``phbase.py:1273-1302`` (``subproblem_creation``),
``phbase.py:803-862`` (``FormEF``) over ``sputils.py:246-383``
(``_create_EF_from_scen_dict``: the scenario objectives weighted by their
probability and normalised by the bundle's, nonanticipativity rows per tree
node), ``phbase.py:985-995`` (feasibility propagated to the bundle's
scenarios) and ``phbase.py:314-354`` (Ebound over subproblems, each with the
bundle's probability).

MI355X form: the bundles of a rank are a second scenario-batched layout
whose "scenario" is a bundle.  Every bundle has the same shape -- T blocks
(T = the largest bundle; a shorter bundle's last block is inert: its columns
fixed at 0, its rows free) of the scenario pattern plus (T - 1) x K
nonanticipativity rows x_t[k] - x_ref[k] = 0, x_ref the bundle's first
scenario at block t's node for slot k (the reference's ref_vars,
sputils.py:350-364: a star per tree node).  Where slot k is at one node for
every scenario (two-stage) the reference is block 0 and the row has two
entries; otherwise the row of block t holds every block 0..t and its values
(per bundle, like every value of the batch) put -1 on the node's first block
of that bundle, 0 on the others.  A row is active when block t is real,
shares the node with an earlier real block and its nonant is not fixed
(nonant_for_fixed_vars=False).  The batched
solver runs on that layout unchanged; its PH terms are gathered from the
scenario arrays with the EF weights p_s / P_b, and its solution is scattered
back to the scenarios' x (``ph_gather`` in include/phgpu.h).
"""
import numpy as np

from .batch import BatchData, NodeInfo


def assign_bundles(rank_slices, all_scenario_names, bundles_per_rank):
    """``spbase.py:206-240``: {rank: {bundle: [scenario names]}}.

    Each rank's scenarios are cut into ``bundles_per_rank`` contiguous
    slices, ``range(int(i*avg), int((i+1)*avg))`` with ``avg = count /
    bundles_per_rank``; more bundles than scenarios is an error."""
    n_proc = len(rank_slices)
    if n_proc * bundles_per_rank > len(all_scenario_names):
        raise RuntimeError("Not enough scenarios to satisfy the bundles_per_rank requirement")
    out = {}
    for rank, slc in enumerate(rank_slices):
        names = [all_scenario_names[i] for i in slc]
        avg = len(names) / bundles_per_rank
        out[rank] = {b: [names[i] for i in range(int(b * avg), int((b + 1) * avg))]
                     for b in range(bundles_per_rank)}
    return out


class BundleLayout:
    """The bundle batch of one rank and its index maps.

    Args:
        data: the rank's scenario :class:`BatchData` (min form).
        groups: per bundle, the local scenario indices in order.
        prob: [S] scenario probabilities.
        gid: [K][S] node-slot ids (``SPBase._create_node_slots``).
        names: bundle names (``"rank{r}bundle{b}"``, phbase.py:1288).

    Attributes (numpy, host): ``data`` (the bundle BatchData), ``term_idx`` /
    ``term_wt`` [Kb*Sb] (bundle PH-term slot -> flat index k*S + s of the
    scenario arrays, weight p_s / P_b), ``x_idx`` [n*S] (scenario x element
    -> flat index of the bundle x), ``bundle_of`` [S], ``P`` [Sb].
    """

    def __init__(self, data: BatchData, groups, prob, gid, names):
        S, n, m, K = data.S, data.n, data.m, data.K
        Sb = len(groups)
        T = max(len(g) for g in groups)
        if min(len(g) for g in groups) < 1:
            raise RuntimeError("an empty bundle")
        self.T, self.Sb, self.names = T, Sb, list(names)
        prob = np.asarray(prob, dtype=np.float64)
        member = np.full((T, Sb), S, dtype=np.int64)      # S: the inert block
        for b, g in enumerate(groups):
            member[:len(g), b] = g
        real = member < S
        P = np.array([prob[g].sum() for g in groups])
        wt = np.where(real, np.append(prob, 0.0)[member] / P[None, :], 0.0)   # [T][Sb]
        self.member, self.P, self.wt = member, P, wt
        bundle_of = np.empty(S, dtype=np.int64)
        pos_of = np.empty(S, dtype=np.int64)
        for b, g in enumerate(groups):
            bundle_of[g] = b
            pos_of[g] = np.arange(len(g))
        self.bundle_of, self.pos_of = bundle_of, pos_of
        # -- pattern: T diagonal blocks, then the (T-1) x K link rows
        nb = T * n
        nc = data.nonant_cols.astype(np.int64)
        rp, ci = data.row_ptr.astype(np.int64), data.col_idx.astype(np.int64)
        nnz = ci.size
        row_ptr = [rp[:-1] + t * nnz for t in range(T)]
        col_idx = [ci + t * n for t in range(T)]
        base = T * nnz
        L = (T - 1) * K
        # slot k's link rows: the reference block is block 0 (the bundle's
        # first scenario) when every scenario has slot k at the same node
        # (two-stage): entries (0, t); else the node's first block in the
        # bundle, which differs by bundle: entries (0 .. t), values per bundle
        star = np.all(gid == gid[:, :1], axis=1) if S > 0 else np.ones(K, dtype=bool)
        gext = np.concatenate([gid, np.full((K, 1), -1)], axis=1)
        fixed = np.concatenate([data.l[nc] == data.u[nc], np.ones((K, 1), dtype=bool)], axis=1)  # [K][S+1]
        lcols, lvals, lptr = [], [], [0]
        lrl = np.full((T - 1, K, Sb), -np.inf)
        for t in range(1, T):
            gt = gext[:, member[t]]                                   # [K][Sb] block t's node
            # the node's first real block before t (-1: none)
            ref = np.full((K, Sb), -1, dtype=np.int64)
            for tp in range(t - 1, -1, -1):
                hit = real[tp][None, :] & (gext[:, member[tp]] == gt)
                ref = np.where(hit, tp, ref)
            ref = np.where(star[:, None], np.where(real[0][None, :] & (gext[:, member[0]] == gt), 0, -1), ref)
            on = real[t][None, :] & (ref >= 0) & ~fixed[:, member[t]]
            lrl[t - 1] = np.where(on, 0.0, -np.inf)
            for k in range(K):
                blocks = [0, t] if star[k] else list(range(t + 1))
                lcols.extend(bk * n + nc[k] for bk in blocks)
                v = np.zeros((len(blocks), Sb))
                v[-1] = 1.0
                for q, bk in enumerate(blocks[:-1]):
                    v[q] = np.where(ref[k] == bk, -1.0, 0.0)
                lvals.append(v)
                lptr.append(lptr[-1] + len(blocks))
        row_ptr.append(base + np.asarray(lptr[:-1], dtype=np.int64))
        col_idx.append(np.asarray(lcols, dtype=np.int64))
        row_ptr = np.concatenate(row_ptr + [[base + lptr[-1]]])
        col_idx = np.concatenate(col_idx)
        mb = T * m + L
        # -- values and data (an extra zero / inert column per array for the pad)
        def take(a, fill):
            ext = np.concatenate([a, np.full((a.shape[0], 1), fill)], axis=1)
            return np.concatenate([ext[:, member[t]] for t in range(T)], axis=0)
        vals = np.concatenate([take(data.vals, 0.0)] + lvals, axis=0)
        c = np.concatenate([np.concatenate([data.c, np.zeros((n, 1))], axis=1)[:, member[t]] * wt[t][None, :]
                            for t in range(T)], axis=0)
        const = (np.append(data.const, 0.0)[member] * wt).sum(axis=0)
        lb = take(data.l, 0.0)
        ub = take(data.u, 0.0)
        rl = take(data.rl, -np.inf)
        ru = take(data.ru, np.inf)
        # link rows: active when block t is real and shares slot k's node with
        # an earlier real block, and its nonant is not fixed in its scenario
        # (the bundle EF is formed with nonant_for_fixed_vars=False,
        # phbase.py:860-861, sputils.py:358-360: no row for a fixed Var; a
        # fixed reference still anchors the others)
        lru = np.where(np.isfinite(lrl), 0.0, np.inf)
        rl = np.concatenate([rl, lrl.reshape(L, Sb)], axis=0)
        ru = np.concatenate([ru, lru.reshape(L, Sb)], axis=0)
        nonant_b = (np.arange(T)[:, None] * n + nc[None, :]).reshape(-1)
        Kb = T * K
        self.data = BatchData(list(names), row_ptr, col_idx, vals, c, const, lb, ub, rl, ru,
                              nonant_b, [NodeInfo([("BUNDLE", 1.0, Kb)])] * Sb, data.sense,
                              prob=P, var_names=None)
        assert self.data.m == mb and self.data.n == nb
        # -- index maps for ph_gather
        k_of = np.tile(np.arange(K), T)                    # bundle slot -> k
        t_of = np.repeat(np.arange(T), K)                  # bundle slot -> block
        mem = member[t_of]                                 # [Kb][Sb]
        self.term_idx = np.where(mem < S, k_of[:, None] * S + mem, -1).astype(np.int32).reshape(-1)
        self.term_wt = wt[t_of].reshape(-1)
        jb = pos_of[None, :] * n + np.arange(n)[:, None]   # [n][S] bundle row of element (j, s)
        self.x_idx = (jb * Sb + bundle_of[None, :]).astype(np.int64)
        if self.x_idx.max(initial=0) >= 2 ** 31 or self.term_idx.size >= 2 ** 31:
            raise RuntimeError("bundle layout too large for int32 gather indices")
        self.x_idx = self.x_idx.astype(np.int32).reshape(-1)


class BundleView:
    """``local_subproblems[bname]`` of a bundled run: the bundle's name, its
    scenarios (``scen_list``, phbase.py:1295-1296) and probability
    (``_mpisppy_probability``, phbase.py:1297-1298)."""

    def __init__(self, name, scen_list, prob):
        self.name = name
        self.scen_list = list(scen_list)
        self._ef_scenario_names = self.scen_list
        self._mpisppy_probability = float(prob)
