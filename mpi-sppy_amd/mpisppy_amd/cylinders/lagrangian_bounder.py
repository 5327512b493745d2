"""Lagrangian outer bound on the batched GPU solver
(mirrors ``mpisppy/cylinders/lagrangian_bounder.py``).

The spoke's per-W work -- ``solve_loop`` with W on and no prox, then
``Ebound`` with a serial-number check (``lagrangian_bounder.py:19-53``) -- runs
as one batched LP launch on the same kernels as the PH hub.  W reaches the
spoke either as flat lists (``main(W_stream)``, ``localWs``) or, inside the
in-process wheel (``cylinders/hub.py``), as a device-to-device copy of the
hub's W tensor (``hub_sync``) in place of the reference's RMA windows
(``spoke.py:59-99``).

Asynchronous (``launch`` / ``harvest``): the spoke's batch runs on a HIP
stream of its own; ``launch`` copies the hub's W (the hub's stream waits for
that copy only) and queues the LP solves, which then overlap the hub's next
PH iterations; ``harvest`` at the next sync waits for them and forms the
bound with the serial-number check -- the reference's spokes likewise report
a bound computed from an earlier W (``spoke.py:59-111``, write ids).
"""
import torch

from .hub import spoke_stream


class LagrangianOuterBound:
    converger_spoke_char = "L"
    bound_kind = "outer"

    def __init__(self, opt, cylinder_size=1):
        self.opt = opt
        self.localWs = None
        self.serial_number = 0
        self.cylinder_size = cylinder_size
        self.bound = None
        self.trivial_bound = None

    def get_serial_number(self):
        return self.serial_number

    def lagrangian_prep(self):
        """lagrangian_bounder.py:9-17: PH_Prep(attach_prox=False), W on, solvers."""
        verbose = self.opt.options["verbose"]
        self.opt.PH_Prep(attach_prox=False)
        self.opt._reenable_W()
        self.opt.subproblem_creation(verbose)
        self.opt._create_solvers()

    def lagrangian(self):
        """lagrangian_bounder.py:19-57: batched LP solves + Ebound (serial check)."""
        verbose = self.opt.options["verbose"]
        self.opt.solve_loop(
            solver_options=self.opt._bound_solver_options(self.opt.current_solver_options),
            dtiming=False,
                            gripe=True, tee=False, verbose=verbose)
        serial_number = self.get_serial_number()
        bound, extra_sums = self.opt.Ebound(verbose, extra_sum_terms=[serial_number])
        serial_number_sum = int(round(extra_sums[0]))
        total = int(self.opt.n_proc) * serial_number
        if total == serial_number_sum:
            return bound
        if self.opt.cylinder_rank == 0:
            print("WARNING: Lagrangian spokes out of sync")
        return None

    def _set_weights_and_solve(self):
        self.opt.W_from_flat_list(self.localWs)
        return self.lagrangian()

    def main(self, W_stream=()):
        """Trivial bound, then one bound per W vector from ``W_stream``
        (an iterable of (serial_number, flat local W) pairs)."""
        self.lagrangian_prep()
        self.trivial_bound = self.lagrangian()
        self.bound = self.trivial_bound
        for serial, Ws in W_stream:
            self.serial_number = serial
            self.localWs = Ws
            b = self._set_weights_and_solve()
            if b is not None:
                self.bound = b
        return self.bound

    # ---- in-process wheel (cylinders/hub.py)
    def spoke_init(self):
        self.opt._own_stream = True
        self.lagrangian_prep()
        with spoke_stream(self.opt):
            self.trivial_bound = self.lagrangian()
        self.bound = self.trivial_bound
        self.in_flight = False

    def launch(self, hub_opt):
        """Queue a bound at the hub's current W: the W copy (the hub's stream
        waits for it), then the batched LP solves; returns at once."""
        with spoke_stream(self.opt):
            self.opt.W.copy_(hub_opt.W)
            ev = torch.cuda.Event() if self.opt.W.is_cuda else None
            if ev is not None:
                ev.record()
            self.serial_number += 1
            self._kw = self.opt.solve_loop_launch(
                solver_options=self.opt._bound_solver_options(self.opt.current_solver_options))
        if ev is not None:
            torch.cuda.current_stream(self.opt.W.device).wait_event(ev)
        self.in_flight = True

    def harvest(self):
        """Wait for the launched solves, then Ebound with the serial check."""
        with spoke_stream(self.opt):
            self.opt.solve_loop_finish(self._kw, gripe=True)
            b = self._ebound_checked()
        self.in_flight = False
        if b is not None and (self.bound is None or
                              (b > self.bound if self.opt.is_minimizing else b < self.bound)):
            self.bound = b
        return b

    def _ebound_checked(self):
        verbose = self.opt.options["verbose"]
        serial_number = self.get_serial_number()
        bound, extra_sums = self.opt.Ebound(verbose, extra_sum_terms=[serial_number])
        if int(self.opt.n_proc) * serial_number == int(round(extra_sums[0])):
            return bound
        if self.opt.cylinder_rank == 0:
            print("WARNING: Lagrangian spokes out of sync")
        return None

    def hub_sync(self, hub_opt):
        """The hub's current W (device copy, same local scenarios), then a
        bound (blocking: launch + harvest)."""
        self.launch(hub_opt)
        return self.harvest()

    def finalize(self):
        self.final_bound = self._set_weights_and_solve()
        self.bound = self.final_bound
        return self.final_bound
