"""Lagrangian outer bound on the batched GPU solver
(mirrors ``mpisppy/cylinders/lagrangian_bounder.py``).

The spoke's per-W work -- ``solve_loop`` with W on and no prox, then
``Ebound`` with a serial-number check (``lagrangian_bounder.py:19-53``) -- runs
as one batched LP launch on the same kernels as the PH hub.  W reaches the
spoke either as flat lists (``main(W_stream)``, ``localWs``) or, inside the
in-process wheel (``cylinders/hub.py``), as a device-to-device copy of the
hub's W tensor (``hub_sync``) in place of the reference's RMA windows
(``spoke.py:59-99``).
"""


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
        self.lagrangian_prep()
        self.trivial_bound = self.lagrangian()
        self.bound = self.trivial_bound

    def hub_sync(self, hub_opt):
        """The hub's current W (device copy, same local scenarios), then a bound."""
        self.opt.W.copy_(hub_opt.W)
        self.serial_number += 1
        b = self.lagrangian()
        if b is not None and (self.bound is None or
                              (b > self.bound if self.opt.is_minimizing else b < self.bound)):
            self.bound = b
        return b

    def finalize(self):
        self.final_bound = self._set_weights_and_solve()
        self.bound = self.final_bound
        return self.final_bound
