"""Xhat shuffle inner-bound spoke (``mpisppy/cylinders/xhatshufflelooper_bounder.py``).

Each sync takes the hub's current nonant values (device copy), tries the
next scenario of a seeded shuffle as xhat (``XhatBase._try_one``, one
batched fixed-nonant LP solve) and reports the best inner bound so far
(``xhatshufflelooper_bounder.py:112-190``).  Two-stage problems.
"""
import numpy as np
import torch

from ..extensions.xhatbase import XhatBase


class XhatShuffleInnerBound:
    converger_spoke_char = "X"
    bound_kind = "inner"

    def __init__(self, opt, seed=42, tries_per_sync=1):
        self.opt = opt
        self.seed = seed
        self.tries_per_sync = tries_per_sync
        self.best = None
        self.best_scenario = None

    def spoke_init(self):
        opt = self.opt
        opt.PH_Prep(attach_duals=False, attach_prox=False)
        opt.subproblem_creation(opt.options.get("verbose", False))
        opt._create_solvers()
        if len(opt.all_nodenames) > 1:
            raise NotImplementedError("the xhat shuffle spoke covers two-stage problems")
        names = list(opt.all_scenario_names)
        np.random.RandomState(self.seed).shuffle(names)
        self.order = names
        self.next = 0
        self.xb = XhatBase(opt)

    def hub_sync(self, hub_opt):
        """Nonants from the hub, then the next shuffled candidate(s)."""
        cols = torch.as_tensor(hub_opt.batch_data.nonant_cols.astype(np.int64), device=hub_opt.device)
        xs = self.opt.batch.x.view(self.opt.batch.n, self.opt.S_loc)
        xh = hub_opt.batch.x.view(hub_opt.batch.n, hub_opt.S_loc)
        xs[cols] = xh.index_select(0, cols)
        for _ in range(self.tries_per_sync):
            sname = self.order[self.next % len(self.order)]
            self.next += 1
            obj = self.xb._try_one({"ROOT": sname})
            if obj is not None and (self.best is None or
                                    (obj < self.best if self.opt.is_minimizing else obj > self.best)):
                self.best, self.best_scenario = obj, sname
        return self.best
