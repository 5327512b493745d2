"""Xhat shuffle inner-bound spoke (``mpisppy/cylinders/xhatshufflelooper_bounder.py``).

Each sync takes the hub's current nonant values (device copy), tries the
next scenario of a seeded shuffle as xhat (``XhatBase._try_one``, one
batched fixed-nonant LP solve) and reports the best inner bound so far
(``xhatshufflelooper_bounder.py:112-190``).  Two-stage problems.

Asynchronous (``launch`` / ``harvest``, see cylinders/hub.py): the spoke's
batch runs on its own stream; ``launch`` copies the hub's nonants (the hub's
stream waits for the copy only) and queues the candidate's fixed-nonant
solve, ``harvest`` evaluates it at the next sync.
"""
import numpy as np
import torch

from ..extensions.xhatbase import XhatBase
from .hub import spoke_stream


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
        opt._own_stream = True
        self.in_flight = False
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

    def _copy_nonants(self, hub_opt):
        """The hub's nonant values into this spoke's x (on the spoke's
        stream; the hub's stream waits for the copy)."""
        cols = torch.as_tensor(hub_opt.batch_data.nonant_cols.astype(np.int64), device=hub_opt.device)
        with spoke_stream(self.opt):
            xs = self.opt.batch.x.view(self.opt.batch.n, self.opt.S_loc)
            xh = hub_opt.batch.x.view(hub_opt.batch.n, hub_opt.S_loc)
            xs[cols] = xh.index_select(0, cols)
            ev = torch.cuda.Event() if xs.is_cuda else None
            if ev is not None:
                ev.record()
        if ev is not None:
            torch.cuda.current_stream(xs.device).wait_event(ev)

    def _keep(self, obj, sname):
        if obj is not None and (self.best is None or
                                (obj < self.best if self.opt.is_minimizing else obj > self.best)):
            self.best, self.best_scenario = obj, sname

    def hub_sync(self, hub_opt):
        """Nonants from the hub, then the next shuffled candidate(s) (blocking)."""
        self._copy_nonants(hub_opt)
        with spoke_stream(self.opt):
            for _ in range(self.tries_per_sync):
                sname = self.order[self.next % len(self.order)]
                self.next += 1
                self._keep(self.xb._try_one({"ROOT": sname}), sname)
        return self.best

    def launch(self, hub_opt):
        """Nonants from the hub, the next candidate's solve queued."""
        self._copy_nonants(hub_opt)
        with spoke_stream(self.opt):
            self._sname = self.order[self.next % len(self.order)]
            self.next += 1
            self._kw = self.xb._try_one_launch({"ROOT": self._sname})
        self.in_flight = True

    def harvest(self):
        with spoke_stream(self.opt):
            self._keep(self.xb._try_one_finish(self._kw), self._sname)
        self.in_flight = False
        return self.best
