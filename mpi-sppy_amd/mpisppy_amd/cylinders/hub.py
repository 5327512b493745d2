"""PH hub with in-process spokes (``mpisppy/cylinders/hub.py``, ``spoke.py``).

The reference runs each cylinder on its own group of MPI ranks and moves W,
nonants and bounds through RMA windows (``spcommunicator.py:100-127``,
``hub.py:285-368``).  Here every rank runs the hub and every spoke on its
own GPU: each spoke owns a separate device batch of the same local
scenarios, and a sync is a device-to-device copy of the hub's W (to W
spokes) or nonant values (to nonant spokes) followed by the spoke's batched
solve; the bounds come back through the spokes' own allreduces.  The hub's
gap bookkeeping and termination test follow ``hub.py:60-137`` and
``PHHub.is_converged`` (``hub.py:430-466``).  Syncs happen every
``sync_every`` PH iterations.

Asynchronous spokes (``async_spokes``, default on): each spoke's batch runs
on its own HIP stream.  At a sync the hub first harvests what every spoke
launched at the previous sync (waiting only if it is still running), then
launches new work at its current W / nonants -- a device-to-device copy the
hub's stream waits for, then the spoke's solves, which overlap the hub's next
PH iterations on the GPU.  A spoke's bound therefore describes the hub's
state one sync earlier, as a reference spoke's bound describes the W it last
read from its window (``spoke.py:59-111``); the schedule is the same on
every rank, so the spokes' collectives stay matched.  ``hub_finalize``
harvests and then runs one blocking sync at the final state.
"""
import contextlib
import math

import torch

from .. import global_toc


def spoke_stream(opt):
    """Context: torch's current stream becomes the spoke batch's own stream,
    ordered after the caller's current stream (no-op for CPU batches or a
    batch on the default stream)."""
    b = getattr(opt, "batch", None)
    ts = getattr(b, "stream", None) if b is not None else None
    if not isinstance(ts, torch.cuda.Stream):
        return contextlib.nullcontext()
    ts.wait_stream(torch.cuda.current_stream(ts.device))
    return torch.cuda.stream(ts)


class PHHub:
    def __init__(self, opt, spokes=(), options=None, sync_every=1, async_spokes=True):
        self.opt = opt
        self.spokes = list(spokes)
        self.options = dict(options or {})
        self.sync_every = max(1, int(sync_every))
        self.async_spokes = bool(async_spokes)
        self.global_rank = opt.cylinder_rank
        self.print_init = True
        self.latest_ib_char = None
        self.latest_ob_char = None
        if opt.is_minimizing:
            self.BestInnerBound, self.BestOuterBound = math.inf, -math.inf
        else:
            self.BestInnerBound, self.BestOuterBound = -math.inf, math.inf
        self.has_outerbound_spokes = any(getattr(s, "bound_kind", "") == "outer" for s in self.spokes)
        self.has_innerbound_spokes = any(getattr(s, "bound_kind", "") == "inner" for s in self.spokes)
        opt.spcomm = self
        self._last_sync = None

    # ------------------------------------------------------------ bounds --
    def OuterBoundUpdate(self, new_bound, char="*"):
        """hub.py:139-160."""
        if new_bound is None:
            return self.BestOuterBound
        better = new_bound > self.BestOuterBound if self.opt.is_minimizing \
            else new_bound < self.BestOuterBound
        if better:
            self.BestOuterBound = new_bound
            self.latest_ob_char = char
        return self.BestOuterBound

    def InnerBoundUpdate(self, new_bound, char="*"):
        """hub.py:162-183."""
        if new_bound is None:
            return self.BestInnerBound
        better = new_bound < self.BestInnerBound if self.opt.is_minimizing \
            else new_bound > self.BestInnerBound
        if better:
            self.BestInnerBound = new_bound
            self.latest_ib_char = char
        return self.BestInnerBound

    def compute_gap(self, compute_relative=True):
        """hub.py:65-88."""
        if self.opt.is_minimizing:
            abs_gap = self.BestInnerBound - self.BestOuterBound
        else:
            abs_gap = self.BestOuterBound - self.BestInnerBound
        if (not math.isnan(abs_gap) and not math.isinf(abs_gap)
                and not math.isnan(self.BestOuterBound) and self.BestOuterBound != 0):
            rel_gap = abs_gap / abs(self.BestOuterBound)
        else:
            rel_gap = math.inf
        return rel_gap if compute_relative else abs_gap

    def get_update_string(self):
        if self.latest_ib_char is None and self.latest_ob_char is None:
            return "   "
        if self.latest_ib_char is None:
            return self.latest_ob_char + "  "
        if self.latest_ob_char is None:
            return "  " + self.latest_ib_char
        return self.latest_ob_char + " " + self.latest_ib_char

    def screen_trace(self):
        """hub.py:100-117."""
        it = self.current_iteration()
        rel_gap = self.compute_gap(True)
        abs_gap = self.compute_gap(False)
        if self.print_init:
            global_toc(f'{"Iter.":>5s}  {"   "}  {"Best Bound":>14s}  {"Best Incumbent":>14s}  '
                       f'{"Rel. Gap":>12s}  {"Abs. Gap":>14s}', True)
            self.print_init = False
        global_toc(f"{it:5d}  {self.get_update_string()}  {self.BestOuterBound:14.4f}  "
                   f"{self.BestInnerBound:14.4f}  {rel_gap * 100:12.3f}%  {abs_gap:14.4f}", True)
        self.latest_ib_char = self.latest_ob_char = None

    def determine_termination(self):
        """hub.py:119-137."""
        abs_ok = rel_ok = False
        if "rel_gap" in self.options and self.options["rel_gap"] is not None:
            rel_ok = self.compute_gap(True) <= self.options["rel_gap"]
        if "abs_gap" in self.options and self.options["abs_gap"] is not None:
            abs_ok = self.compute_gap(False) <= self.options["abs_gap"]
        if abs_ok:
            global_toc(f"Terminating based on inter-cylinder absolute gap "
                       f"{self.compute_gap(False):12.4f}", self.global_rank == 0)
        if rel_ok:
            global_toc(f"Terminating based on inter-cylinder relative gap "
                       f"{self.compute_gap(True) * 100:12.3f}%", self.global_rank == 0)
        return abs_ok or rel_ok

    # -------------------------------------------------------------- sync --
    def sync(self):
        """hub.py:417-428: W to W spokes, nonants to nonant spokes, bounds back."""
        if self._last_sync is not None and self.opt._PHIter - self._last_sync < self.sync_every:
            return
        self._last_sync = self.opt._PHIter
        for sp in self.spokes:
            if self.async_spokes and hasattr(sp, "launch"):
                if getattr(sp, "in_flight", False):
                    self._update(sp, sp.harvest())
                sp.launch(self.opt)
            else:
                self._update(sp, sp.hub_sync(self.opt))

    def _update(self, sp, b):
        if sp.bound_kind == "outer":
            self.OuterBoundUpdate(b, sp.converger_spoke_char)
        else:
            self.InnerBoundUpdate(b, sp.converger_spoke_char)

    def sync_with_spokes(self):
        self.sync()

    def is_converged(self):
        """hub.py:430-466."""
        if self.opt._PHIter >= 1 and getattr(self.opt, "trivial_bound", None) is not None:
            self.OuterBoundUpdate(self.opt.trivial_bound)
        if self.opt.options.get("display_progress", False) and self.global_rank == 0:
            self.screen_trace()
        if not self.has_innerbound_spokes:
            return False
        return self.determine_termination()

    def current_iteration(self):
        return self.opt._PHIter

    def main(self):
        """hub.py:468-470: PH with this hub as its spoke communicator."""
        for sp in self.spokes:
            sp.spoke_init()
        return self.opt.ph_main()

    def hub_finalize(self):
        """Final bounds from the spokes at the hub's last W / nonants (what is
        still in flight first)."""
        for sp in self.spokes:
            if getattr(sp, "in_flight", False):
                self._update(sp, sp.harvest())
            self._update(sp, sp.hub_sync(self.opt))
