"""Extensive form of a two-stage or multistage scenario set (TEST INFRASTRUCTURE).

Restates ``mpisppy/utils/sputils.py:_create_EF_from_scen_dict`` (168-383):
probability-weighted scenario objectives, one copy of every scenario's
variables, and non-anticipativity rows x_s[k] == x_ref[k] per tree node.
Solved with HiGHS simplex; used only to pin the oracle against the
reference's published EF values.
"""
import numpy as np
import scipy.sparse as sp

from .solve import _highs_solve


def solve_ef(scens, nonant_for_fixed_vars=True):
    """nonant_for_fixed_vars=False: no row for a fixed (l == u) variable of a
    later scenario (sputils.py:358-360; the reference's bundles, phbase.py:860-861)."""
    S = len(scens)
    prob = np.array([s.prob if s.prob is not None else 1.0 / S for s in scens])
    sgn = 1.0 if scens[0].sense == "min" else -1.0
    ns = [s.A.shape[1] for s in scens]
    offs = np.concatenate([[0], np.cumsum(ns)])
    blocks = [s.A for s in scens]
    A = sp.block_diag(blocks, format="lil")
    rl = list(np.concatenate([s.rl for s in scens]))
    ru = list(np.concatenate([s.ru for s in scens]))
    c = np.concatenate([sgn * p * s.c for p, s in zip(prob, scens)])
    l = np.concatenate([s.l for s in scens])
    u = np.concatenate([s.u for s in scens])
    rows = []
    first = {}
    for si, s in enumerate(scens):
        for (nm, cp, idx) in s.nodes:
            if nm not in first:
                first[nm] = (si, idx)
                continue
            r0, ridx = first[nm]
            for a, b in zip(idx, ridx):
                if not nonant_for_fixed_vars and s.l[a] == s.u[a]:
                    continue
                rows.append(((si, a), (r0, b)))
    na = sp.lil_matrix((len(rows), int(offs[-1])))
    for r, ((si, a), (r0, b)) in enumerate(rows):
        na[r, offs[si] + a] = 1.0
        na[r, offs[r0] + b] = -1.0
        rl.append(0.0)
        ru.append(0.0)
    Afull = sp.vstack([A.tocsr(), na.tocsr()]).tocsr()
    status, x, _, _ = _highs_solve(c, None, Afull, np.array(rl), np.array(ru), l, u)
    obj = float(c @ x) + sum(p * sgn * s.const for p, s in zip(prob, scens))
    xs = [x[offs[i]:offs[i + 1]] for i in range(S)]
    return sgn * obj, xs
