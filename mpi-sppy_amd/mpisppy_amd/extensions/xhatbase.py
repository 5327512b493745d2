"""Inner bounds from a candidate first-stage solution (``mpisppy/extensions/xhatbase.py``).

``_try_one(snamedict)`` (xhatbase.py:35-145): every node's nonants are taken
from the scenario ``snamedict[node]`` holds them for (broadcast from its
rank), fixed in every local scenario, and the scenarios are re-solved with W
and prox off (one batched LP solve on the GPU: the nonant columns' bounds
are set to l = u = xhat through ``ph_batch_set_bounds``).  If every scenario
solves, the expected objective is an inner bound (an upper bound for
minimisation); the nonants' previous values and bounds are restored.

Infeasibility: the batched PDHG does not certify primal infeasibility, so a
scenario that does not reach the tolerance within ``xhat_max_iters`` counts
as infeasible for the candidate (the bound is then None, as the reference
returns for infeasible candidates).
"""
import numpy as np
import torch


class XhatBase:
    def __init__(self, opt):
        self.opt = opt
        self.cylinder_rank = opt.cylinder_rank
        self.n_proc = opt.n_proc
        self.verbose = opt.options.get("verbose", False)

    def _xhat_from(self, snamedict):
        """Dense [G] vector of node-slot values: node nd's nonants from the
        scenario snamedict[nd] (summed over ranks: only its owner adds)."""
        opt = self.opt
        xg = np.zeros(opt.G)
        have = np.zeros(opt.G)
        x = opt.batch.x.view(opt.batch.n, opt.S_loc)
        cols = opt.batch_data.nonant_cols
        pos = {nm: i for i, nm in enumerate(opt.local_scenario_names)}
        for nd, sname in snamedict.items():
            if nd not in opt.node_offset:
                raise RuntimeError(f"{nd} is not a tree node")
            s = pos.get(sname)
            if s is None:
                continue
            off = 0
            for (name, cp, nlen) in opt.batch_data.node_infos[s].nodes:
                if name == nd:
                    base = opt.node_offset[nd]
                    vals = x[torch.as_tensor(cols[off:off + nlen].astype(np.int64),
                                             device=x.device), s].cpu().numpy()
                    xg[base:base + nlen] = vals
                    have[base:base + nlen] = 1.0
                    break
                off += nlen
            else:
                raise RuntimeError(f"scenario {sname} does not pass through node {nd}")
        tot = opt.comm.allreduce_host(list(np.concatenate([xg, have])))
        tot = np.asarray(tot)
        xg, have = tot[:opt.G], tot[opt.G:]
        for nd in opt.node_offset:
            base, nlen = opt.node_offset[nd], opt.node_nlen[nd]
            if np.any(have[base:base + nlen] != 1.0):
                raise RuntimeError(f"snamedict gives no (or several) scenarios for node {nd}")
        return xg

    def _try_one(self, snamedict, solver_options=None, verbose=False, restore_nonants=True):
        """xhatbase.py:35-145: expected objective at the candidate, or None."""
        kw = self._try_one_launch(snamedict, solver_options)
        return self._try_one_finish(kw, verbose, restore_nonants)

    def _try_one_launch(self, snamedict, solver_options=None):
        """The candidate's nonants fixed and the batched solve queued (not
        waited for; asynchronous spokes).  Returns the solve keywords."""
        opt = self.opt
        xg = self._xhat_from(snamedict)
        opt._save_nonants()
        opt._fix_nonants(xg)
        sopt = dict(solver_options or {})
        sopt.setdefault("pdhg_max_iters", int(opt.options.get("xhat_max_iters", 50000)))
        return opt.solve_loop_launch(solver_options=sopt, dis_W=True, dis_prox=True)

    def _try_one_finish(self, kw, verbose=False, restore_nonants=True):
        """Wait for the candidate's solve; E[objective] or None."""
        opt = self.opt
        opt.solve_loop_finish(kw)
        status = opt.batch.status.cpu().numpy()
        solved = opt.comm.allreduce_host([float(np.sum(status != 0))])[0] == 0.0
        if not solved or opt.infeas_prob() != 0.0:
            opt._restore_nonants()
            return None
        w_dis, p_dis = opt.W_disabled, opt.prox_disabled
        opt._disable_W_and_prox()
        obj = opt.Eobjective(verbose=verbose)
        if not w_dis:
            opt._reenable_W()
        if not p_dis:
            opt._reenable_prox()
        if restore_nonants:
            opt._restore_nonants()
        else:
            opt._unfix_nonants()
        return obj


def xhat_shuffle_inner_bound(opt, tries=None, seed=42, solver_options=None):
    """The shuffle looper's inner bound (cylinders/xhatshufflelooper_bounder.py:
    112-190), two-stage: try scenarios as xhat in a seeded random order and
    keep the best expected objective.  Returns (bound, scenario name) or
    (None, None)."""
    xb = XhatBase(opt)
    names = list(opt.all_scenario_names)
    rng = np.random.RandomState(seed)
    rng.shuffle(names)
    if tries is not None:
        names = names[:tries]
    best, best_name = None, None
    for sname in names:
        obj = xb._try_one({"ROOT": sname}, solver_options=solver_options)
        if obj is None:
            continue
        if best is None or (obj < best if opt.is_minimizing else obj > best):
            best, best_name = obj, sname
    return best, best_name
