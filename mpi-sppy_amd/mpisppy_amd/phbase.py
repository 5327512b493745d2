"""PHBase on the MI355X batched solver (mirrors ``mpisppy/phbase.py``).

Method names, argument meanings, option keys and the Iter0 / iterk_loop
sequencing follow the reference (citations per method).  What changes is
where the work happens:

* ``solve_loop`` issues ONE batched PDHG launch for all local scenarios
  (``ph_pdhg_solve``) instead of ``solve_one`` per scenario;
* W, rho, xbar, xsqbar live in HBM as [K][S] (scenario-fastest) tensors and
  are updated by device kernels; the per-node Allreduce of Compute_Xbar and
  the scalar Allreduces of convergence_diff / Ebound / Eobjective become
  ``torch.distributed`` all_reduce calls (RCCL over xGMI on GPUs).
"""
import math
import time
import warnings

import contextlib
import numpy as np
import torch

from . import SOLVER_NAMES, global_toc
from .spbase import SPBase

# solver option keys understood by the PDHG batch (iter0/iterk_solver_options)
_PDHG_KEYS = {"pdhg_tol": "tol", "pdhg_max_iters": "max_iters",
              "pdhg_check_every": "check_every", "warm_start": "warm_start",
              "pdhg_reflection": "reflection", "pdhg_polish": "polish"}
_DEFAULT_SOLVE = dict(tol=1e-9, max_iters=200000, check_every=64, warm_start=True,
                      reflection=1.0, polish=True)


def _nullctx():
    return contextlib.nullcontext()


class PHBase(SPBase):
    """Base class for PH on the batched GPU solver.  See ``phbase.py:31-142``."""

    def __init__(self, PHoptions, all_scenario_names, scenario_creator,
                 scenario_denouement=None, all_nodenames=None, mpicomm=None,
                 scenario_creator_kwargs=None, PH_extensions=None,
                 PH_extension_kwargs=None, PH_converger=None, rho_setter=None,
                 variable_probability=None):
        super().__init__(PHoptions, all_scenario_names, scenario_creator,
                         scenario_denouement=scenario_denouement,
                         all_nodenames=all_nodenames, mpicomm=mpicomm,
                         scenario_creator_kwargs=scenario_creator_kwargs,
                         variable_probability=variable_probability)
        global_toc("Initializing PHBase", self.options.get("verbose", False))
        self.PHoptions = PHoptions
        self.options_check()
        self.PH_extensions = PH_extensions
        self.PH_extension_kwargs = PH_extension_kwargs
        self.PH_converger = PH_converger
        self.rho_setter = rho_setter
        self.iter0_solver_options = PHoptions["iter0_solver_options"]
        self.iterk_solver_options = PHoptions["iterk_solver_options"]
        self.W_disabled = None
        self.prox_disabled = None
        self.convobject = None
        self.conv = None
        self._PHIter = 0
        self._prox_approx = False
        self._duals_attached = False
        self._prox_attached = False
        self.w_on = 0.0
        self.prox_on = 0.0
        self.batch = None
        self.device = torch.device("cuda", torch.cuda.current_device()) \
            if torch.cuda.is_available() else torch.device("cpu")
        self._warned_keys = set()
        self.solve_log = []   # (n_scenarios, seconds, mean iters, max iters, polished)
        self._alloc_state()
        self.attach_xbars()
        if self.PH_extensions is not None:
            if self.PH_extension_kwargs is None:
                self.extobject = self.PH_extensions(self)
            else:
                self.extobject = self.PH_extensions(self, **self.PH_extension_kwargs)

    # ------------------------------------------------------------- state --
    def _alloc_state(self):
        d = self.batch_data
        dev = self.device
        f64 = dict(dtype=torch.float64, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        K, S = d.K, d.S
        self.K, self.S_loc = K, S
        self.prob = torch.as_tensor(self.local_prob, **f64)
        self.prob_coeff = torch.as_tensor(self.prob_coeff_host.reshape(-1), **f64)
        self.gid = torch.as_tensor(self.gid_host.reshape(-1), **i32)
        self.slot_k = torch.as_tensor(self.slot_k_host, **i32)
        self.slot_s0 = torch.as_tensor(self.slot_s0_host, **i32)
        self.slot_s1 = torch.as_tensor(self.slot_s1_host, **i32)
        self.absdiff = torch.zeros(S, **f64)
        self.obj_buf = torch.zeros(S, **f64)
        self.seg_all = torch.tensor([0, S], **i32)
        self.scal = torch.zeros(1, **f64)
        # variable probabilities (spbase.py:369-400): W mask, or None
        self.w_coeff = None if self.w_coeff_host is None else \
            torch.as_tensor(self.w_coeff_host.reshape(-1), **f64)
        # convergence_diff: the reference's rank slices (ref_n_proc ranks)
        R = int(self.PHoptions.get("ref_n_proc", self.n_proc))
        if R < 1 or R > len(self.all_scenario_names):
            raise ValueError("ref_n_proc must be in [1, number of scenarios]")
        from .utils.sputils import rank_slices
        slices = rank_slices(len(self.all_scenario_names), R)
        # ref slices are contiguous and cover every scenario (S >= R), so the
        # local part of ref slice r is [clamp(start_r), clamp(start_{r+1}))
        seg = [min(max(sl[0], self.local_begin), self.local_end) - self.local_begin
               for sl in slices]
        seg.append(self.local_end - self.local_begin)
        self.ref_n_proc = R
        self.conv_seg = torch.tensor(seg, **i32)
        self.conv_cnt = np.array([max(len(sl), 1) * K for sl in slices], dtype=np.float64)
        # one buffer [xbar sums 2G | conv partials R]: with several ranks the
        # device loop allreduces both in one collective (conv one pass late)
        self.xconv = torch.zeros(2 * self.G + R, **f64)
        self.xsums = self.xconv[:2 * self.G]
        self.conv_parts = self.xconv[2 * self.G:]
        # the device loop's pass (ph_loop_pass) allreduces [2G sums | one
        # pre-weighted conv partial]
        self.xpass = self.xconv[:2 * self.G + 1]
        self.conv_part = self.xconv[2 * self.G:2 * self.G + 1]
        self._one = torch.ones(1, **f64)
        self._x_save = self._y_save = None
        self.conv_cnt_dev = torch.as_tensor(self.conv_cnt, **f64)
        # the same weights per local scenario, 1/cnt[r(s)]/R (fused W + conv)
        wconv = np.zeros(S)
        for r in range(R):
            wconv[seg[r]:seg[r + 1]] = 1.0 / self.conv_cnt[r] / R
        self.conv_w = torch.as_tensor(wconv, **f64)
        self.conv_hist = None
        self._loop_graphs = {}
        self._graphs_failed = False
        self.scenario_feasible = np.ones(S, dtype=bool)
        self._all_feasible = True

    # ---------------------------------------------------------- options --
    def options_check(self):
        """phbase.py:1240-1270."""
        required = ["solvername", "PHIterLimit", "defaultPHrho", "convthresh", "verbose",
                    "display_progress", "iter0_solver_options", "iterk_solver_options"]
        self._options_check(required, self.PHoptions)
        if "display_timing" not in self.PHoptions:
            self.PHoptions["display_timing"] = False
        if "display_convergence_detail" not in self.PHoptions:
            self.PHoptions["display_convergence_detail"] = False
        if self.PHoptions["solvername"] not in SOLVER_NAMES:
            raise ValueError(f"solvername {self.PHoptions['solvername']!r} is not served by "
                             f"mpisppy_amd; use one of {SOLVER_NAMES}")

    def _solve_kwargs(self, solver_options):
        kw = dict(_DEFAULT_SOLVE)
        for k, v in (solver_options or {}).items():
            if k in _PDHG_KEYS:
                kw[_PDHG_KEYS[k]] = v
            elif k not in self._warned_keys:
                self._warned_keys.add(k)
                if self.cylinder_rank == 0:
                    warnings.warn(f"solver option {k}={v} ignored by the PDHG batch solver")
        return kw

    def _bound_solver_options(self, solver_options):
        """Solver options for the bound solves (post_solve_bound, the
        Lagrangian spoke).  The per-scenario bound is the dual objective of
        the returned (x, y); a dual residual on a one-sided column makes it
        exact only up to that residual times |x|, so at the 1e-9 default the
        10k-scenario farmer bound overshot the EF optimum by 3e-8 relative.
        Unless the caller sets ``pdhg_tol``, bound solves run at
        PHoptions["bound_pdhg_tol"] (default 1e-12), which the exact
        active-set polish reaches in FP64."""
        o = dict(solver_options or {})
        o.setdefault("pdhg_tol", self.PHoptions.get("bound_pdhg_tol", 1e-12))
        return o

    # ------------------------------------------------- W / prox attach --
    def attach_xbars(self):
        """phbase.py:1622-1632."""
        f64 = dict(dtype=torch.float64, device=self.device)
        self.xbar = torch.zeros(self.K * self.S_loc, **f64)
        self.xsqbar = torch.zeros(self.K * self.S_loc, **f64)

    def attach_Ws_and_prox(self):
        """phbase.py:1110-1131: W=0, rho=defaultPHrho, both terms disabled."""
        f64 = dict(dtype=torch.float64, device=self.device)
        self.W = torch.zeros(self.K * self.S_loc, **f64)
        self.rho = torch.full((self.K * self.S_loc,), float(self.PHoptions["defaultPHrho"]), **f64)
        self.w_on = 0.0
        self.prox_on = 0.0
        self.W_disabled = True
        self.prox_disabled = True

    def attach_PH_to_objective(self, add_duals=True, add_prox=False):
        """phbase.py:1133-1209 (the terms are formed inside the solve kernel)."""
        if self.PHoptions.get("linearize_proximal_terms", False):
            raise NotImplementedError("linearize_proximal_terms: the GPU solver handles the "
                                      "exact prox QP; linearization is not supported")
        self._duals_attached = bool(add_duals)
        self._prox_attached = bool(add_prox)

    def PH_Prep(self, attach_duals=True, attach_prox=True):
        """phbase.py:1211-1238."""
        self.current_solver_options = self.PHoptions["iter0_solver_options"]
        self.attach_Ws_and_prox()
        self.attach_PH_to_objective(add_duals=attach_duals, add_prox=attach_prox)
        if self.PH_extensions is not None:
            self.extobject.pre_iter0()

    def _set_flags(self):
        self.w_on = 1.0 if (self._duals_attached and not self.W_disabled) else 0.0
        self.prox_on = 1.0 if (self._prox_attached and not self.prox_disabled) else 0.0

    def _disable_prox(self):
        self.prox_disabled = True
        self._set_flags()

    def _disable_W_and_prox(self):
        self.prox_disabled = True
        self.W_disabled = True
        self._set_flags()

    def _disable_W(self):
        self.W_disabled = True
        self._set_flags()

    def _reenable_prox(self):
        self.prox_disabled = False
        self._set_flags()

    def _reenable_W_and_prox(self):
        self.prox_disabled = False
        self.W_disabled = False
        self._set_flags()

    def _reenable_W(self):
        self.W_disabled = False
        self._set_flags()

    def subproblem_creation(self, verbose=False):
        """phbase.py:1273-1302: the subproblems are the scenarios, or with
        bundles_per_rank the bundles (formed at SPBase construction as one
        batched layout, bundles.BundleLayout)."""
        if self.bundling and verbose and self.cylinder_rank == 0:
            for bname, bv in self.local_subproblems.items():
                for sname in bv.scen_list:
                    print("bundling " + sname + " into " + bname)
        self.subproblems_created = True

    def _create_solvers(self):
        """phbase.py:1304-1362: SolverFactory + set_instance  ->  ONE device batch."""
        if self.batch is not None:
            return
        from .batch import DeviceBatch
        t0 = time.time()
        stream = None
        if getattr(self, "_own_stream", False) and self.device.type == "cuda":
            # a spoke's batch: its kernels on a stream of their own, so they
            # overlap the hub's (cylinders/hub.py, asynchronous spokes)
            stream = torch.cuda.Stream(self.device)
            stream.wait_stream(torch.cuda.current_stream(self.device))
        self.batch = DeviceBatch(self.batch_data, device=self.device, stream=stream)
        if self.bundling:
            self._create_bundle_batch(stream)
        self.set_instance_time = time.time() - t0

    def _create_bundle_batch(self, stream, batch_factory=None):
        """Bundles (phbase.py:1273-1302, 803-862): the rank's bundle
        subproblems as a second device batch (bundles.BundleLayout) with the
        index maps of its PH-term gather and solution scatter.
        (batch_factory: a test's CPU stand-in instead of DeviceBatch.)"""
        from .batch import DeviceBatch
        bl = self.bundle_layout
        dev = self.device
        self.bbatch = DeviceBatch(bl.data, device=dev, stream=stream) if batch_factory is None \
            else batch_factory(bl.data)
        f64 = dict(dtype=torch.float64, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        self._b_term_idx = torch.as_tensor(bl.term_idx, **i32)
        self._b_term_wt = torch.as_tensor(bl.term_wt, **f64)
        self._b_x_idx = torch.as_tensor(bl.x_idx, **i32)
        nt = bl.term_idx.size
        self._b_W = torch.zeros(nt, **f64)
        self._b_rho = torch.zeros(nt, **f64)
        self._b_xbar = torch.zeros(nt, **f64)
        self._b_prob = torch.as_tensor(bl.P, **f64)
        self._b_seg = torch.tensor([0, bl.Sb], **i32)
        self._b_of = torch.as_tensor(bl.bundle_of, dtype=torch.int64, device=dev)
        self._b_scal = torch.zeros(1, **f64)

    def _launch_solve(self, kw, use_scenarios=False):
        """Queue the batched solve of every local subproblem.  With bundles:
        the bundle batch's PH terms gathered from the scenario arrays with
        the EF weights p_s / P_b, the bundle solve, and its solution
        scattered to the scenarios' x (the scenario sub-blocks hold the EF
        solution, phbase.py:833-838); one ph_gather call per array.
        ``use_scenarios``: solve_loop's use_scenarios_not_subproblems
        (phbase.py:1038-1041): the scenario batch even when bundling."""
        self._solved_scenarios = use_scenarios or not self.bundling
        if self._solved_scenarios:
            self.batch.solve(self.W, self.rho, self.xbar, self.w_on, self.prox_on, **kw)
            return
        bb = self.bbatch
        nt = self._b_term_idx.numel()
        for src, dst, wt in ((self.W, self._b_W, self._b_term_wt), (self.rho, self._b_rho, self._b_term_wt),
                             (self.xbar, self._b_xbar, None)):
            bb.gather(src, self._b_term_idx, wt, nt, dst)
        bb.solve(self._b_W, self._b_rho, self._b_xbar, self.w_on, self.prox_on, **kw)
        bb.gather(bb.x, self._b_x_idx, None, self._b_x_idx.numel(), self.batch.x)

    def _solve_summary(self):
        """(not optimal, PDHG iterations sum, max, polished, cached) of the
        last solve (waits for it); with bundles the bundle solve's, and the
        bundle statuses copied to their scenarios (phbase.py:992-995)."""
        if getattr(self, "_solved_scenarios", True):
            return self.batch.summary()
        out = self.bbatch.summary()
        ts = getattr(self.batch, "torch_stream", None)
        with torch.cuda.stream(ts) if ts is not None else _nullctx():
            self.batch.status.copy_(self.bbatch.status.index_select(0, self._b_of))
        if ts is not None:  # host reads of batch.status (on the current stream) after the copy
            torch.cuda.current_stream(self.device).wait_stream(ts)
        return out

    @property
    def n_subproblems(self):
        return self.S_loc if getattr(self, "_solved_scenarios", True) else self.bundle_layout.Sb

    # ----------------------------------------------------------- solves --
    def solve_loop_launch(self, solver_options=None, dis_W=False, dis_prox=False):
        """The device half of solve_loop: the batched solve is queued on the
        batch's stream and not waited for (asynchronous spokes).  Returns the
        solve keywords for solve_loop_finish."""
        if dis_W and dis_prox:
            self._disable_W_and_prox()
        elif dis_W:
            self._disable_W()
        elif dis_prox:
            self._disable_prox()
        if self.batch is None:
            self._create_solvers()
        kw = self._solve_kwargs(solver_options)
        self._launch_t0 = time.perf_counter()
        self._launch_solve(kw)
        # (the flags were read at launch)
        if dis_W and dis_prox:
            self._reenable_W_and_prox()
        elif dis_W:
            self._reenable_W()
        elif dis_prox:
            self._reenable_prox()
        return kw

    def solve_loop_finish(self, kw, gripe=False):
        """The host half of solve_loop: wait for the solve, statuses ->
        scenario_feasible (phbase.py:959-989)."""
        nonopt, it_sum, it_max, npol, ncache = self._solve_summary()  # waits for the solve
        dt = time.perf_counter() - self._launch_t0
        ns = self.n_subproblems
        self.solve_log.append((ns, dt, it_sum / max(ns, 1), it_max, npol + ncache))
        self._set_feasibility(nonopt, gripe, kw["max_iters"])

    def solve_loop(self, solver_options=None, use_scenarios_not_subproblems=False,
                   dtiming=False, dis_W=False, dis_prox=False, gripe=False,
                   disable_pyomo_signal_handling=False, tee=False, verbose=False):
        """phbase.py:999-1095: one batched solve of every local subproblem."""
        if dis_W and dis_prox:
            self._disable_W_and_prox()
        elif dis_W:
            self._disable_W()
        elif dis_prox:
            self._disable_prox()
        if self.batch is None:
            self._create_solvers()
        kw = self._solve_kwargs(solver_options)
        t0 = time.perf_counter()
        self._launch_solve(kw, use_scenarios=use_scenarios_not_subproblems)
        nonopt, it_sum, it_max, npol, ncache = self._solve_summary()  # waits for the solve
        dt = time.perf_counter() - t0
        ns = self.n_subproblems
        self.solve_log.append((ns, dt, it_sum / max(ns, 1), it_max, npol + ncache))
        self._set_feasibility(nonopt, gripe, kw["max_iters"])
        if dtiming:
            allt = self.comm.allgather_object(dt)
            if self.cylinder_rank == 0:
                print("Pyomo solve times (seconds):")
                print("\tmin=%4.2f mean=%4.2f max=%4.2f" % (np.min(allt), np.mean(allt), np.max(allt)))
        if self.PH_extensions is not None and hasattr(self.extobject, "post_solve_loop"):
            self.extobject.post_solve_loop()
        if dis_W and dis_prox:
            self._reenable_W_and_prox()
        elif dis_W:
            self._reenable_W()
        elif dis_prox:
            self._reenable_prox()

    def _set_feasibility(self, nonopt, gripe, max_iters):
        """phbase.py:959-989: scenario_feasible from the per-scenario
        statuses.  As in the reference, only a solve that ends infeasible or
        unbounded makes the scenario infeasible: statuses 2 / 3 carry a
        primal / dual infeasibility certificate (a Farkas ray of the PDHG
        iterates, csrc/phgpu.hip ray_status).  A solve stopped at the PDHG
        iteration limit (status 1, a solver's iteration limit in the
        reference) keeps its iterate, is griped about, and reports a safe
        Lagrangian dual bound (possibly -inf) as its outer bound; the xhat
        inner bound requires status 0 (extensions/xhatbase.py)."""
        if nonopt:
            status = self.batch.status.cpu().numpy()
            self.scenario_feasible = status <= 1
            sub_names = self.local_scenario_names
            if not getattr(self, "_solved_scenarios", True):  # the reference gripes per subproblem (phbase.py:959-978)
                status = self.bbatch.status.cpu().numpy()
                sub_names = self.bundle_layout.names
        elif not self._all_feasible:
            self.scenario_feasible = np.ones(self.S_loc, dtype=bool)
        self._all_feasible = not nonopt
        if not (gripe and nonopt):
            return
        name = type(self).__name__
        if self.spcomm is not None:
            name = type(self.spcomm).__name__
        why = {2: "primal infeasible (certificate)", 3: "dual infeasible, unbounded (certificate)"}
        what = "scenario" if getattr(self, "_solved_scenarios", True) else "bundle"
        # the reference prints one line per infeasible / unbounded solve
        # (phbase.py:959-978); a batch of 10k scenarios prints the first few
        # and a count (all of them with verbose)
        bad = np.nonzero(status >= 2)[0]
        show = bad if self.PHoptions.get("verbose", False) else bad[:5]
        for i in show:
            print(f"[{name}] Solve failed for {what} {sub_names[i]}: "
                  f"{why.get(int(status[i]), 'status %d' % status[i])}")
        if len(show) < len(bad):
            print(f"[{name}] ... {len(bad) - len(show)} more failed solves "
                  f"({len(bad)} of {len(status)} local {what}s)")
        # an iteration-limit stop is silent in the reference (a solver's
        # maxIterations termination loads its point as feasible): a count
        # with verbose only
        nlim = int(np.sum(status == 1))
        if nlim and self.PHoptions.get("verbose", False):
            print(f"[{name}] {nlim} of {len(status)} local {what}s stopped at the PDHG iteration "
                  f"limit ({max_iters}) short of the KKT tolerance (kept as feasible, safe outer bound)")

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    # ---------------------------------------- nonanticipativity updates --
    def _allreduce(self, t):
        """Collective on a device tensor, ordered on the batch's stream (the
        library's kernels run there; under RCCL the collective is queued on
        torch's current stream)."""
        ts = getattr(self.batch, "torch_stream", None)
        if ts is None or not t.is_cuda or torch.cuda.is_current_stream_capturing():
            # (under graph capture: the capture stream, which the batch's
            # launches also use, so the collective is a node of the graph)
            return self.comm.allreduce_(t)
        with torch.cuda.stream(ts):
            return self.comm.allreduce_(t)

    def Compute_Xbar(self, verbose=False):
        """phbase.py:144-221: weighted node sums, Allreduce, broadcast."""
        b = self.batch
        b.xbar_accum(self.prob_coeff, self.slot_k, self.slot_s0, self.slot_s1, self.xsums)
        self._allreduce(self.xsums)
        b.update_w(self.xsums, self.G, self.gid, self.rho, None, self.xbar, self.xsqbar,
                   None, self.absdiff)
        if verbose and self.cylinder_rank == 0:
            print("xbar:", self.xsums[:self.G].cpu().numpy())

    def Update_W(self, verbose):
        """phbase.py:224-251: W += rho*(x - xbar) (masked by w_coeff if set)."""
        self.batch.update_w(self.xsums, self.G, self.gid, self.rho, self.w_coeff, self.xbar,
                            self.xsqbar, self.W, self.absdiff)

    def convergence_diff(self):
        """phbase.py:254-276: sum over ranks of mean |x - xbar|, / n_proc.

        Reproduces the reference's rank slicing for ``ref_n_proc`` ranks
        (default: this run's rank count)."""
        self.batch.segment_sum(self.absdiff, None, self.conv_seg, self.conv_parts)
        self._allreduce(self.conv_parts)
        parts = self.conv_parts.cpu().numpy()
        return float(np.sum(parts / self.conv_cnt) / self.ref_n_proc)

    def _weighted_sum(self, v):
        self.batch.segment_sum(v, self.prob, self.seg_all, self.scal)
        return self.scal

    def Eobjective(self, verbose=False):
        """phbase.py:279-312: sum_s p_s * (active objective at the current x)."""
        b = self.batch
        b.eval_objective(self.W, self.rho, self.xbar, self.w_on, self.prox_on, self.obj_buf)
        self.obj_buf.add_(b.const)
        t = self._weighted_sum(self.obj_buf).clone()
        self._allreduce(t)
        v = float(t.item())
        return v if self.is_minimizing else -v

    def _outer_bounds(self):
        ob = self.batch.dbound + self.batch.const
        return ob if self.is_minimizing else -ob

    def Ebound(self, verbose=False, extra_sum_terms=None):
        """phbase.py:314-354: sum over subproblems of probability x
        outer_bound (+ extra terms); a bundle's probability is the sum of its
        scenarios' (phbase.py:1297-1298).  After a solve_loop over the
        scenarios themselves (use_scenarios_not_subproblems) the scenarios'
        bounds."""
        if not getattr(self, "_solved_scenarios", True):
            bb = self.bbatch
            ob = bb.dbound + bb.const
            ob = (ob if self.is_minimizing else -ob).contiguous()
            bb.segment_sum(ob, self._b_prob, self._b_seg, self._b_scal)
            t = self._b_scal.clone()
        else:
            ob = self._outer_bounds().contiguous()
            t = self._weighted_sum(ob).clone()
        if extra_sum_terms is not None:
            t = torch.cat([t, torch.tensor(list(extra_sum_terms), dtype=torch.float64,
                                           device=t.device)])
        self._allreduce(t)
        v = t.cpu().numpy()
        if extra_sum_terms is None:
            return float(v[0])
        return float(v[0]), v[1:]

    def _update_E1(self):
        """phbase.py:619-636."""
        self.E1 = self.comm.allreduce_host([float(np.sum(self.local_prob))])[0]

    def feas_prob(self):
        """phbase.py:649-668."""
        return self.comm.allreduce_host(
            [float(np.sum(self.local_prob[self.scenario_feasible]))])[0]

    def infeas_prob(self):
        return self.comm.allreduce_host(
            [float(np.sum(self.local_prob[~self.scenario_feasible]))])[0]

    # ------------------------------------------- fixed-nonant solves --
    def _save_nonants(self):
        """phbase.py:464-486 _save_nonants: the current nonant values of
        every local scenario (device copy).  With bundles the scenario x
        holds the bundle solution (scattered back after every bundle solve),
        so the same copy serves both batches."""
        cols = torch.as_tensor(self.batch_data.nonant_cols.astype(np.int64), device=self.device)
        self._saved_nonant_cols = cols
        self._saved_nonants = self.batch.x.view(self.batch.n, self.S_loc).index_select(0, cols).clone()

    def _bundle_nonant_index(self):
        """Bundle-batch flat indices of every (nonant slot, scenario) element,
        [K][S] (the solution scatter's x_idx restricted to the nonant
        columns)."""
        if getattr(self, "_b_nonant_idx", None) is None:
            cols = torch.as_tensor(self.batch_data.nonant_cols.astype(np.int64), device=self.device)
            S = self.S_loc
            flat = (cols[:, None] * S + torch.arange(S, device=self.device)[None, :]).reshape(-1)
            self._b_nonant_idx = self._b_x_idx.to(torch.int64).index_select(0, flat)
        return self._b_nonant_idx

    def _fix_nonants(self, xhat_slots):
        """phbase.py:514-549 _fix_nonants: every local scenario's nonants
        fixed at the node-slot values xhat_slots [G] (l = u on the nonant
        columns).  With bundles the reference fixes the scenarios' Vars,
        which live in the bundle EFs: the same values go to the bundle
        batch's nonant columns of every block (its solve_loop then solves the
        bundles with those nonants fixed)."""
        b = self.batch
        n, S = b.n, self.S_loc
        vals = torch.as_tensor(np.asarray(xhat_slots, dtype=np.float64)[self.gid_host],
                               device=self.device)               # [K][S]
        cols = torch.as_tensor(self.batch_data.nonant_cols.astype(np.int64), device=self.device)
        l = b.l.clone().view(n, S)
        u = b.u.clone().view(n, S)
        l[cols] = vals
        u[cols] = vals
        b.set_bounds(l.reshape(-1), u.reshape(-1))
        x = b.x.view(n, S)
        x[cols] = vals   # the warm start sits on the fixed values
        if self.bundling:
            bb = self.bbatch
            idx = self._bundle_nonant_index()
            v = vals.reshape(-1)
            bl = bb.l.clone().reshape(-1)
            bu = bb.u.clone().reshape(-1)
            bl[idx] = v
            bu[idx] = v
            bb.set_bounds(bl, bu)
            bb.x.view(-1)[idx] = v

    def _unfix_nonants(self):
        self.batch.set_bounds(self.batch.l, self.batch.u)
        if self.bundling:
            self.bbatch.set_bounds(self.bbatch.l, self.bbatch.u)

    def _restore_nonants(self):
        """phbase.py:488-512 _restore_nonants: saved nonant values back,
        bounds freed (both batches when bundling)."""
        self._unfix_nonants()
        if getattr(self, "_saved_nonants", None) is not None:
            x = self.batch.x.view(self.batch.n, self.S_loc)
            x[self._saved_nonant_cols] = self._saved_nonants
            if self.bundling:
                self.bbatch.x.view(-1)[self._bundle_nonant_index()] = self._saved_nonants.reshape(-1)

    # ---------------------------------------------------------- W I/O --
    def W_from_flat_list(self, flat_list):
        """phbase.py:601-617: flat list in (scenario, nonant) order."""
        a = np.asarray(flat_list, dtype=np.float64).reshape(self.S_loc, self.K)
        self.W.copy_(torch.as_tensor(a.T.reshape(-1), device=self.device))

    def get_flat_W(self):
        """Local W as a flat (scenario, nonant)-ordered numpy array."""
        return self.W.view(self.K, self.S_loc).cpu().numpy().T.reshape(-1)

    def _local_nonant_values(self):
        x = self.batch.x.view(self.batch.n, self.S_loc)
        cols = torch.as_tensor(self.batch_data.nonant_cols.astype(np.int64), device=self.device)
        return x.index_select(0, cols).cpu().numpy()

    def gather_var_values_to_rank0(self, get_zero_prob_values=False):
        """spbase.py:519-543: {(scenario_name, nonant var name): value} on
        rank 0; zero-probability nonants give None unless asked for."""
        vals = self._local_nonant_values()
        names = self.nonant_names()
        zero = np.zeros_like(self.prob_coeff_host, dtype=bool) if self.w_coeff_host is None \
            else (self.prob_coeff_host == 0.0)
        local = {(sn, names[k]): (None if zero[k, s] and not get_zero_prob_values
                                  else float(vals[k, s]))
                 for s, sn in enumerate(self.local_scenario_names) for k in range(self.K)}
        allv = self.comm.gather_object(local)
        if self.cylinder_rank != 0:
            return None
        out = {}
        for d in allv:
            out.update(d)
        return out

    def report_var_values_at_rank0(self, header="", print_zero_prob_values=False):
        v = self.gather_var_values_to_rank0()
        if self.cylinder_rank == 0:
            print(header)
            for (sn, vn), val in sorted(v.items()):
                print(f"  {sn:>20s} {vn:>30s} {val:.6f}")

    def _use_rho_setter(self, verbose):
        """phbase.py:556-588: rho_setter(scenario) -> [(var, rho)] per
        scenario; var is a nonant VarData of the scenario's model, its id()
        (the reference's form) or a nonant variable name (batched scenarios
        without per-scenario models get their ScenarioView)."""
        if self.rho_setter is None:
            return
        models = self.batch_data.models
        rho = self.rho.view(self.K, self.S_loc)
        views = list(self.local_scenarios.values())
        for s in range(self.S_loc):
            target = models[s] if models is not None else views[s]
            for key, r in self.rho_setter(target):
                rho[self._nonant_slot_of(s, key, "rho_setter"), s] = float(r)

    # ----------------------------------------------------------- drivers --
    def Iter0(self):
        """phbase.py:1364-1470."""
        verbose = self.PHoptions["verbose"]
        dprogress = self.PHoptions["display_progress"]
        dtiming = self.PHoptions["display_timing"]
        self._PHIter = 0
        global_toc("Creating solvers", verbose)
        self._create_solvers()
        global_toc("Entering solve loop in PHBase.Iter0", verbose)
        self.solve_loop(solver_options=self.current_solver_options, dtiming=dtiming,
                        gripe=True, verbose=verbose)
        self._update_E1()
        if abs(1 - self.E1) > self.E1_tolerance:
            raise RuntimeError(f"Total probability of scenarios was {self.E1} "
                               f"(E1_tolerance = {self.E1_tolerance})")
        feasP = self.feas_prob()
        if feasP != self.E1:  # phbase.py:1421-1427 (the reference quit()s)
            raise RuntimeError(f"Infeasibility detected; E_feas, E1= {feasP} {self.E1} "
                               "(a scenario is infeasible or was not solved to tolerance)")
        if self.PH_extensions is not None:
            self.extobject.post_iter0()
        if self.rho_setter is not None:
            self._use_rho_setter(verbose and self.cylinder_rank == 0)
        if self.PH_converger is not None:
            self.convobject = self.PH_converger(self)
        self.conv = None
        self.trivial_bound = self.Ebound(verbose)
        if dprogress and self.cylinder_rank == 0:
            print("")
            print("After PH Iteration", self._PHIter)
            print("Trivial bound =", self.trivial_bound)
            print("PHBase Convergence Metric =", self.conv)
            print("Elapsed time: %6.2f" % (time.perf_counter() - self.start_time))
        if self.PHoptions["display_convergence_detail"]:
            self.report_var_values_at_rank0(header="Convergence detail:")
        self._reenable_W_and_prox()
        self.current_solver_options = self.PHoptions["iterk_solver_options"]
        return self.trivial_bound

    # ------------------------------------------------- device-side loop --
    def _device_loop_ok(self):
        """The iterk_loop body can run without a host round trip per iteration
        when nothing on the host has to see each iteration (no extensions,
        converger, hub/spoke communicator or per-iteration printing)."""
        o = self.PHoptions
        return (o.get("device_loop", True) and self.PH_extensions is None and not self.bundling
                and self.PH_converger is None
                and (self.spcomm is None or hasattr(self.spcomm, "sync_every"))
                and not o["display_progress"] and not o["display_convergence_detail"]
                and not o.get("display_timing", False))

    def _device_iteration(self, kw):
        """One iterk_loop pass queued on the device (phbase.py:1498-1553 order):
        Compute_Xbar -> Update_W -> convergence_diff -> [stop?] -> solve, as
        ONE library call (ph_loop_pass, bound by run_device_loop).
        Compute_Xbar's local sums of this pass were computed by the previous
        pass's post-solve kernel (or before the first pass); Compute_Xbar's
        broadcast and Update_W are one kernel, which writes what the two
        reference calls write.  Several ranks: one collective per pass
        before it carries this pass's node sums and the previous pass's
        (pre-weighted) convergence partial; the previous pass's convergence
        test runs inside the call and, if it stops, the host restores the
        x/y saved before that pass's solve (run_device_loop)."""
        if self._pass_collective():
            self._allreduce(self.xpass)
        self.batch.loop_pass()

    def _device_chunk(self, kw, chunk):
        """`chunk` passes.  One rank: ONE library call (ph_loop_run: a
        persistent launch that keeps the scenarios' data in LDS across the
        passes when the batch qualifies, else the per-pass kernels); several
        ranks: one ph_loop_pass per pass after its allreduce."""
        if not self._pass_collective():
            self.batch.loop_run(chunk)
        else:
            for _ in range(chunk):
                self._device_iteration(kw)

    def _bind_pass(self, kw):
        """ph_loop_bind_pass: the device loop's per-pass arguments, once."""
        b = self.batch
        saves = None
        if self._pass_collective():
            if self._x_save is None:
                self._x_save = torch.empty_like(b.x)
                self._y_save = torch.empty_like(b.y)
                self._st_save = torch.empty_like(b.status)
                self._db_save = torch.empty_like(b.dbound)
            saves = (self._x_save, self._y_save, self._st_save, self._db_save)
        b.loop_bind_pass(self.xsums, self.G, self.gid, self.rho, self.w_coeff, self.xbar,
                         self.xsqbar, self.W, self.absdiff, self.conv_w, self.conv_hist,
                         self.conv_part if self._pass_collective() else None, saves,
                         self.w_on, self.prox_on, **kw)

    def run_device_loop(self, start_iter, iter_limit, convthresh, chunk=None):
        """Run iterk_loop passes start_iter+1 .. iter_limit on the device,
        queued `chunk` at a time; the stop flag (convergence or the limit) is
        read once per chunk.  Returns (stop, last iteration)."""
        if self.batch is None:
            self._create_solvers()
        kw = self._solve_kwargs(self.current_solver_options)
        b = self.batch
        chunk = int(chunk or self.PHoptions.get("device_loop_chunk", 64))
        if self.conv_hist is None or self.conv_hist.numel() < max(iter_limit, 1):
            old = self.conv_hist
            size = max(iter_limit, 1024, 0 if old is None else 2 * old.numel())
            self.conv_hist = torch.zeros(size, dtype=torch.float64, device=self.device)
            if old is not None:
                self.conv_hist[:old.numel()] = old
            self._loop_graphs = {}  # captured pointers changed
        b.loop_reset(start_iter, iter_limit, convthresh)
        b.loop_enable(True)
        b.loop_set_xbar(self.prob_coeff, self.slot_k, self.slot_s0, self.slot_s1, self.xsums)
        self._bind_pass(kw)
        # Compute_Xbar's local sums for the first pass
        b.xbar_accum(self.prob_coeff, self.slot_k, self.slot_s0, self.slot_s1, self.xsums)
        graph = None
        if self._graph_ok():
            key = (self.w_on, self.prox_on, tuple(sorted(kw.items())), chunk)
            graph = self._loop_graphs.get(key)
            if graph is None:
                graph = self._capture_chunk(kw, chunk)
                if graph is not None:
                    self._loop_graphs[key] = graph
        try:
            while True:
                t0 = time.perf_counter()
                if graph is not None:
                    graph.replay()
                else:
                    self._device_chunk(kw, chunk)
                st = b.loop_status()
                dt = time.perf_counter() - t0
                stop, it, nonopt, nsolves, it_sum, it_max, npol, ncache = st
                npol += ncache
                prev = getattr(self, "_loop_prev", (0, 0))
                self._loop_prev = (nsolves, npol)
                if nsolves > prev[0]:
                    self.solve_log.append((nsolves - prev[0], dt, it_sum / max(nsolves, 1),
                                           it_max, npol - prev[1]))
                if stop:
                    break
            if self._pass_collective():
                # the last pass's conv partial (limit reached), then the
                # reference's state at a convergence break: x/y of before the
                # solve that the lagged test showed should not have run
                self._allreduce(self.conv_part)
                b.loop_conv_lagged(self.conv_part, self._one, 1.0, self.conv_hist)
                st = b.loop_status()
                stop, it = st[0], st[1]
                nonopt = nonopt or st[2]
                if stop == 1 and self._x_save is not None:
                    # the reference's state at its break: x/y, statuses and
                    # outer bounds of the last solve it ran (the cached
                    # active-set maps stay valid: they depend on the active
                    # set, not on the point)
                    b.x.copy_(self._x_save)
                    b.y.copy_(self._y_save)
                    b.status.copy_(self._st_save)
                    b.dbound.copy_(self._db_save)
                    nonopt = int((b.status != 0).sum().item())
        finally:
            b.loop_enable(False)
            b.loop_set_xbar(None, None, None, None, None)
            b.loop_unbind_pass()
            self._loop_prev = (0, 0)
        self._set_feasibility(nonopt, True, kw["max_iters"])
        return stop, it

    def _pass_collective(self):
        """The several-ranks form of a device-loop pass (one collective of the
        node sums + the lagged convergence partial before each ph_loop_pass):
        several ranks, or the option device_loop_collective (one rank running
        that form, for tests of its capture)."""
        return self.comm.size > 1 or bool(self.PHoptions.get("device_loop_collective", False))

    def _graph_ok(self):
        """Replay chunks of the device loop as one HIP graph (option
        device_loop_graphs: True / False / "auto", the default: graphs only
        for several ranks on RCCL, whose collectives are captured with the
        passes).  One rank:  With one ph_loop_pass call per iteration
        the eager loop issues in ~21 us against ~60 us of GPU work per F2
        iteration, and measured faster than the graph replay
        (profiles/r03: 0.0601 / 0.0612 against 0.0629 / 0.0658 ms per step).
        Replay of mid-size and big-path chunks is EXPERIMENTAL: round 2's
        intermittent mid-size replay fault was not caught in the act (its
        presumed cause, the chunked summary's stop race, was removed and
        device-side checks now turn a recurrence into PH_EDEV),
        so keep the option off outside tests and measurements."""
        b = self.batch
        if self._graphs_failed or self.device.type != "cuda" or not hasattr(b, "set_stream"):
            return False
        opt = self.PHoptions.get("device_loop_graphs", "auto")
        coll = self._pass_collective()
        if coll and self.comm.size > 1 and self.comm.backend != "nccl":
            return False   # (gloo stages collectives through the host: not capturable)
        if opt == "auto":
            # several ranks on RCCL: the pass is a collective + one library
            # call, each a host round trip of ~10-20 us against ~50 us of GPU
            # work at F2, so the chunk is replayed as one graph with the
            # collectives captured on the batch's stream -- for one-wave
            # batches (n + m <= 63) only: mid-size and big chunks stay eager
            # (their replay is the experimental path above, and their passes
            # are milliseconds long, so the host's round trips do not show)
            return coll and self.comm.size > 1 and b.n + b.m <= 63
        return bool(opt)

    def _capture_chunk(self, kw, chunk):
        """Capture `chunk` device iterations (the library's launches moved to
        the capture stream) into a torch.cuda.CUDAGraph."""
        b = self.batch
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(self.device)
        try:
            with torch.cuda.graph(g):
                b.set_stream(torch.cuda.current_stream(self.device).cuda_stream)
                try:
                    for _ in range(chunk):  # (the per-pass kernels and collectives: one graph)
                        self._device_iteration(kw)
                finally:
                    b.set_stream(b.stream_handle)
        except RuntimeError as e:
            # (a capture the runtime refuses -- e.g. a collective library
            # without stream capture -- leaves the eager passes, which are
            # the same computation; nothing of the failed capture ran)
            self._graphs_failed = True
            if self.cylinder_rank == 0:
                print(f"device loop: graph capture failed ({e}); eager passes")
            torch.cuda.synchronize(self.device)
            return None
        return g

    def iterk_loop(self):
        """phbase.py:1472-1566: Xbar -> W -> conv -> [hub] -> break? -> solve."""
        if self._device_loop_ok():
            max_iterations = int(self.PHoptions["PHIterLimit"])
            thresh = float(self.PHoptions["convthresh"])
            if self.spcomm is None:
                stop, it = self.run_device_loop(0, max_iterations, thresh)
            else:
                # hub: device-loop chunks of sync_every iterations, the spokes
                # synced and the gap tested between chunks (phbase.py:1517-1521)
                every = int(self.spcomm.sync_every)
                stop, it = 0, 0
                while it < max_iterations:
                    stop, it = self.run_device_loop(it, min(it + every, max_iterations), thresh,
                                                    chunk=every)
                    self._PHIter = it
                    if stop == 1:
                        break
                    self.spcomm.sync()
                    if self.spcomm.is_converged():
                        global_toc("Cylinder convergence", self.cylinder_rank == 0)
                        break
            self._PHIter = it
            hist = self.conv_hist[:it].cpu().numpy() if it > 0 else np.zeros(0)
            self.conv_history = [float(v) for v in hist]
            self.conv = self.conv_history[-1] if it > 0 else None
            if stop == 1:
                global_toc("Convergence metric=%f dropped below user-supplied threshold=%f"
                           % (self.conv, self.PHoptions["convthresh"]),
                           self.cylinder_rank == 0 and self.PHoptions["verbose"])
            return
        verbose = self.PHoptions["verbose"]
        have_extensions = self.PH_extensions is not None
        have_converger = self.PH_converger is not None
        dprogress = self.PHoptions["display_progress"]
        dtiming = self.PHoptions["display_timing"]
        self.conv = None
        max_iterations = int(self.PHoptions["PHIterLimit"])
        self.conv_history = []
        for self._PHIter in range(1, max_iterations + 1):
            iteration_start_time = time.time()
            if dprogress:
                global_toc(f"\nInitiating PH Iteration {self._PHIter}\n", self.cylinder_rank == 0)
            self.Compute_Xbar(verbose)
            self.Update_W(verbose)
            self.conv = self.convergence_diff()
            self.conv_history.append(self.conv)
            if have_extensions:
                self.extobject.miditer()
            if self.spcomm is not None:
                self.spcomm.sync()
                if self.spcomm.is_converged():
                    global_toc("Cylinder convergence", self.cylinder_rank == 0)
                    break
            if have_converger:
                if self.convobject.is_converged():
                    global_toc("User-supplied converger determined termination criterion reached",
                               self.cylinder_rank == 0)
                    break
            elif self.conv is not None:
                if self.conv < self.PHoptions["convthresh"]:
                    global_toc("Convergence metric=%f dropped below user-supplied threshold=%f"
                               % (self.conv, self.PHoptions["convthresh"]),
                               self.cylinder_rank == 0 and (verbose or dprogress))
                    break
            self.solve_loop(solver_options=self.current_solver_options, dtiming=dtiming,
                            gripe=True, verbose=verbose)
            if have_extensions:
                self.extobject.enditer()
            if dprogress and self.cylinder_rank == 0:
                print("")
                print("After PH Iteration", self._PHIter)
                print("Scaled PHBase Convergence Metric=", self.conv)
                print("Iteration time: %6.2f" % (time.time() - iteration_start_time))
                print("Elapsed time:   %6.2f" % (time.perf_counter() - self.start_time))
            if self.PHoptions["display_convergence_detail"]:
                self.report_var_values_at_rank0(header="Convergence detail:")
            if self._PHIter == max_iterations:
                global_toc("Reached user-specified limit=%d on number of PH iterations"
                           % max_iterations, self.cylinder_rank == 0 and (verbose or dprogress))

    def post_loops(self, PH_extensions=None):
        """phbase.py:1568-1620."""
        dprogress = self.PHoptions["display_progress"]
        self.comm.Barrier()
        if self.scenario_denouement is not None:
            for sname, s in self.local_scenarios.items():
                self.scenario_denouement(self.cylinder_rank, sname, s)
        self.comm.Barrier()
        if PH_extensions is not None:
            self.extobject.post_everything()
        Eobj = self.Eobjective(self.PHoptions["verbose"])
        self.comm.Barrier()
        if dprogress and self.cylinder_rank == 0:
            print("")
            print("Current ***weighted*** E[objective] =", Eobj)
            print("")
        return Eobj

    def post_solve_bound(self, solver_options=None, verbose=False):
        """phbase.py:753-801: W on, prox off, LP solves, Ebound."""
        if self.cylinder_rank == 0:
            print("Warning: Lagrangian bounds might not be correct in certain "
                  "cases where there are integers not subject to "
                  "non-anticipativity and those integers do not reach integrality.")
        if self.W_disabled:
            self._reenable_W()
        self._disable_prox()
        self.solve_loop(solver_options=self._bound_solver_options(solver_options),
                        dis_prox=False, gripe=True,
                        tee=False, verbose=verbose)
        bound = self.Ebound(verbose)
        self._reenable_prox()
        return bound

    # ----------------------------------------------------------- metrics --
    def solves_per_second(self):
        """Scenario subproblem solves per second of solve_loop wall time (local)."""
        n = sum(x[0] for x in self.solve_log)
        t = sum(x[1] for x in self.solve_log)
        return n / t if t > 0 else math.nan
