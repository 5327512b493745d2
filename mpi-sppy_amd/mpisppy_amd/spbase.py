"""Scenario distribution and tree bookkeeping (mirrors ``mpisppy/spbase.py``).

Keeps the reference's data semantics -- contiguous rank slices
(``spbase.py:172-203`` -> ``sputils.py:619-628``), uniform default
probabilities (``spbase.py:486-490``), ``prob_coeff[node] = p_s /
uncond_prob(node)`` (``spbase.py:353-366``) and the nonant order
(``scenario_tree.py:36``) -- but stores the local scenarios as ONE
scenario-batched layout (:mod:`mpisppy_amd.batch`) instead of a dict of
Pyomo models.
"""
import time

import numpy as np

from . import global_toc
from .batch import BatchData, from_models
from .comm import Comm
from .utils import sputils


class ScenarioView:
    """What ``local_scenarios[name]`` gives back: the scenario's name, model
    (when built per scenario), probability and tree path."""

    def __init__(self, spb, idx):
        self._spb = spb
        self._idx = idx
        self.name = spb.local_scenario_names[idx]
        self._mpisppy_probability = float(spb.local_prob[idx])
        self._mpisppy_node_names = [nd[0] for nd in spb.batch_data.node_infos[idx].nodes]
        models = spb.batch_data.models
        self.model = None if models is None else models[idx]

    def nonant_values(self):
        return self._spb._local_nonant_values()[:, self._idx]


class SPBase:
    """Base class: distributes scenarios and builds the batched layout.

    Args mirror ``SPBase.__init__`` (``spbase.py:42-53``).  ``mpicomm`` is a
    torch.distributed process group (or :class:`Comm`); ``None`` means the
    default group when torch.distributed is initialised, else one rank.
    ``scenario_creator`` may carry a ``batch_creator(names, **kwargs)``
    attribute that builds the local batch without per-scenario models.
    """

    def __init__(self, options, all_scenario_names, scenario_creator,
                 scenario_denouement=None, all_nodenames=None, mpicomm=None,
                 scenario_creator_kwargs=None, variable_probability=None,
                 E1_tolerance=1e-5):
        self.start_time = time.perf_counter()
        self.options = options
        self.all_scenario_names = list(all_scenario_names)
        self.scenario_creator = scenario_creator
        self.scenario_denouement = scenario_denouement
        self.E1_tolerance = E1_tolerance
        self.variable_probability = variable_probability
        if all_nodenames is None:
            self.all_nodenames = ["ROOT"]
        elif "ROOT" in all_nodenames:
            self.all_nodenames = list(all_nodenames)
        else:
            raise RuntimeError("'ROOT' must be in the list of node names")
        self.multistage = len(self.all_nodenames) > 1
        self.comm = Comm.wrap(mpicomm)
        self.mpicomm = self.comm
        self.cylinder_rank = self.comm.rank
        self.n_proc = self.comm.size
        self.global_rank = self.comm.rank
        global_toc("Initializing SPBase")
        if self.n_proc > len(self.all_scenario_names):
            raise RuntimeError("More ranks than scenarios")
        self.names_in_bundles = None
        self.bundling = int(options.get("bundles_per_rank", 0) or 0) > 0  # spbase.py:206 (> 0)
        if "branching_factors" in options:
            self.branching_factors = options["branching_factors"]
        else:
            self.branching_factors = [len(self.all_scenario_names)]
        self._calculate_scenario_ranks()
        if self.bundling:
            self._assign_bundles()
        self._create_scenarios(scenario_creator_kwargs)
        self._look_and_leap()
        self._compute_unconditional_node_probabilities()
        self._create_node_slots()
        self._verify_nonant_lengths()
        self.is_minimizing = self.batch_data.sense == "min"
        self._use_variable_probability_setter(options.get("verbose", False))
        self.bundle_layout = self._form_bundles() if self.bundling else None
        self._spcomm = None

    # ---------------------------------------------------------------- setup
    def _calculate_scenario_ranks(self):
        self._rank_slices, self._scenario_slices = sputils.scen_names_to_ranks(
            self.all_scenario_names, self.n_proc)
        self.local_scenario_indices = self._rank_slices[self.cylinder_rank]
        self.local_scenario_names = [self.all_scenario_names[i] for i in self.local_scenario_indices]
        self.local_begin = self.local_scenario_indices[0]
        self.local_end = self.local_scenario_indices[-1] + 1

    def _assign_bundles(self):
        """spbase.py:206-240: names_in_bundles[rank][bundle] = [scenario names]."""
        from .bundles import assign_bundles
        bpr = int(self.options["bundles_per_rank"])
        if self.options.get("verbose", False) and self.cylinder_rank == 0:
            print("(rank0)", bpr, "bundles per rank")
        self.names_in_bundles = assign_bundles(self._rank_slices, self.all_scenario_names, bpr)

    def _form_bundles(self):
        """phbase.py:1273-1302 + 803-862: this rank's bundles as ONE batched
        layout of bundle subproblems (:class:`bundles.BundleLayout`)."""
        from .bundles import BundleLayout
        idx = {nm: i for i, nm in enumerate(self.local_scenario_names)}
        mine = self.names_in_bundles[self.cylinder_rank]
        groups = [[idx[nm] for nm in mine[b]] for b in sorted(mine)]
        names = [f"rank{self.cylinder_rank}bundle{b}" for b in sorted(mine)]
        return BundleLayout(self.batch_data, groups, self.local_prob, self.gid_host, names)

    def _create_scenarios(self, scenario_creator_kwargs):
        kw = {} if scenario_creator_kwargs is None else dict(scenario_creator_kwargs)
        t0 = time.time()
        bc = getattr(self.scenario_creator, "batch_creator", None)
        if bc is not None and not self.options.get("per_scenario_models", False):
            data = bc(self.local_scenario_names, **kw)
        else:
            models = [self.scenario_creator(nm, **kw) for nm in self.local_scenario_names]
            data = from_models(self.local_scenario_names, models)
        if not isinstance(data, BatchData):
            raise TypeError("batch_creator must return a BatchData")
        self.batch_data = data
        self.instance_creation_time = time.time() - t0
        self.scenarios_constructed = True

    def _look_and_leap(self):
        d = self.batch_data
        if d.prob is None:
            prob = 1.0 / len(self.all_scenario_names)
            if self.cylinder_rank == 0 and self.options.get("verbose", False):
                print(f"Did not find _mpisppy_probability, assuming uniform probability {prob}")
            self.local_prob = np.full(d.S, prob)
        else:
            self.local_prob = np.asarray(d.prob, dtype=np.float64)

    def _compute_unconditional_node_probabilities(self):
        """prob_coeff per (nonant slot, scenario), spbase.py:353-366."""
        d = self.batch_data
        pc = np.zeros((d.K, d.S))
        for s, ni in enumerate(d.node_infos):
            unc = 1.0
            off = 0
            for j, (name, cp, nlen) in enumerate(ni.nodes):
                unc = 1.0 if j == 0 else unc * cp
                pc[off:off + nlen, s] = self.local_prob[s] / unc
                off += nlen
        self.prob_coeff_host = pc

    def _create_node_slots(self):
        """Global node-slot numbering for the dense xbar buffer.

        slot g = (node, i) for every node in ``all_nodenames`` order; a rank
        holding no scenario of a node contributes zeros to its sums, so one
        allreduce equals the reference's per-node communicators.
        """
        d = self.batch_data
        local_nlen = {}
        for ni in d.node_infos:
            for (name, cp, nlen) in ni.nodes:
                if name not in self.all_nodenames:
                    raise RuntimeError(f"Tree node '{name}' not in all_nodenames list {self.all_nodenames}")
                if local_nlen.setdefault(name, nlen) != nlen:
                    raise RuntimeError(f"node {name} has inconsistent nonant lengths")
        lens = [local_nlen.get(nm, -1) for nm in self.all_nodenames]
        glens = self.comm.allreduce_host(lens, op="max")
        self.node_nlen = {nm: int(v) for nm, v in zip(self.all_nodenames, glens)}
        for nm, v in self.node_nlen.items():
            if v < 0:
                raise RuntimeError(f"no scenario references tree node {nm}")
        self.node_offset = {}
        g = 0
        for nm in self.all_nodenames:
            self.node_offset[nm] = g
            g += self.node_nlen[nm]
        self.G = g
        K, S = d.K, d.S
        gid = np.zeros((K, S), dtype=np.int32)
        slot_k = np.zeros(g, dtype=np.int32)
        slot_s0 = np.zeros(g, dtype=np.int32)
        slot_s1 = np.zeros(g, dtype=np.int32)
        seen = {}
        for s, ni in enumerate(d.node_infos):
            off = 0
            for (name, cp, nlen) in ni.nodes:
                base = self.node_offset[name]
                gid[off:off + nlen, s] = base + np.arange(nlen)
                if name in seen:
                    first_s, koff, last_s = seen[name]
                    if koff != off:
                        raise RuntimeError(f"node {name} sits at different nonant offsets")
                    if last_s != s - 1:
                        raise RuntimeError(f"scenarios of node {name} are not contiguous")
                    seen[name] = (first_s, koff, s)
                else:
                    seen[name] = (s, off, s)
                off += nlen
        for name, (s0, koff, s1) in seen.items():
            base = self.node_offset[name]
            for i in range(self.node_nlen[name]):
                slot_k[base + i] = koff + i
                slot_s0[base + i] = s0
                slot_s1[base + i] = s1 + 1
        self.gid_host = gid
        self.slot_k_host, self.slot_s0_host, self.slot_s1_host = slot_k, slot_s0, slot_s1

    def _nonant_slot_of(self, s, key, who="variable_probability"):
        """Nonant slot k of scenario s named by ``key``: a nonant VarData of
        the scenario's model, ``id()`` of one (the reference's form,
        ``spbase.py:386-388``), or a nonant variable name.  ``who`` names the
        caller in the error messages (variable_probability, rho_setter)."""
        d = self.batch_data
        if not hasattr(self, "_slot_by_name"):
            names = self.nonant_names()
            self._slot_by_name = {nm: k for k, nm in enumerate(names)}
            self._col2slot = {int(c): k for k, c in enumerate(d.nonant_cols)}
        if isinstance(key, str):
            if key not in self._slot_by_name:
                raise KeyError(f"{who}: {key!r} is not a nonant")
            return self._slot_by_name[key]
        models = d.models
        if models is None:
            raise TypeError(f"{who}: without per-scenario models, name nonants "
                            "by variable name")
        mdl = models[s]
        from . import repn
        if isinstance(key, int):
            ids = getattr(mdl, "_mpisppy_amd_nonant_ids", None)
            if ids is None:
                ids = {}
                for node in mdl._mpisppy_node_list:
                    for vd in node.nonant_vardata_list:
                        ids[id(vd)] = self._col2slot[repn.column_of(mdl, vd)]
                mdl._mpisppy_amd_nonant_ids = ids
            if key not in ids:
                raise KeyError(f"{who}: id is not a nonant of the scenario")
            return ids[key]
        col = repn.column_of(mdl, key)
        if col not in self._col2slot:
            raise KeyError(f"{who}: variable is not a nonant")
        return self._col2slot[col]

    def _use_variable_probability_setter(self, verbose=False):
        """spbase.py:369-400: per-variable probabilities.

        ``variable_probability(scenario, **variable_probability_kwargs)``
        returns [(var, prob)] for the scenario (var: VarData, its id(), or a
        nonant name).  The probability REPLACES prob_coeff of that nonant
        (so Compute_Xbar weights it), and a zero probability masks the
        nonant's W (``w_coeff``, applied by Update_W, phbase.py:246-251).
        As in the reference, touching any nonant of a tree node turns the
        whole node into per-variable values (defaults kept for the rest)."""
        d = self.batch_data
        self.w_coeff_host = None
        self.has_variable_probability = self.variable_probability is not None
        if self.variable_probability is None:
            return
        kw = self.options.get("variable_probability_kwargs", dict())
        wc = np.ones((d.K, d.S))
        didit = 0
        for s, (sname, view) in enumerate(self.local_scenarios.items()):
            target = view.model if view.model is not None else view
            for key, prob in self.variable_probability(target, **kw):
                k = self._nonant_slot_of(s, key)
                self.prob_coeff_host[k, s] = float(prob)
                if prob == 0:
                    wc[k, s] = 0.0
                didit += 1
        self.w_coeff_host = wc
        if verbose and self.cylinder_rank == 0:
            print("variable_probability set", didit, "and skipped", d.K * d.S - didit)
        if "do_not_check_variable_probabilities" in self.options \
                and not self.options["do_not_check_variable_probabilities"]:
            self._check_variable_probabilities_sum(verbose)

    def _check_variable_probabilities_sum(self, verbose):
        """spbase.py:417-460: per node slot, the sum of prob_coeff over all
        scenarios of the node must be 1 (within E1_tolerance)."""
        d = self.batch_data
        sums = np.zeros(self.G)
        np.add.at(sums, self.gid_host.reshape(-1), self.prob_coeff_host.reshape(-1))
        tot = np.asarray(self.comm.allreduce_host(sums.tolist()))
        bad = np.nonzero(~np.isclose(tot, 1.0, atol=self.E1_tolerance))[0]
        if bad.size:
            names = self.nonant_names()
            slot_of_g = {int(g): int(k) for k, g in zip(np.repeat(np.arange(d.K), d.S),
                                                         self.gid_host.reshape(-1))}
            raise RuntimeError("Node conditional probabilities do not sum to 1 for nonants "
                               + ", ".join(f"{names[slot_of_g[g]]} (sum {tot[g]})" for g in bad))
        if verbose and self.cylinder_rank == 0:
            print("Checked variable probability sums")

    def is_zero_prob(self, scenario_model, var):
        """spbase.py:402-415."""
        if self.variable_probability is None:
            return False
        s = self.local_scenario_names.index(scenario_model.name)
        return float(self.prob_coeff_host[self._nonant_slot_of(s, var), s]) == 0.0

    def _verify_nonant_lengths(self):
        ks = self.comm.allreduce_host([self.batch_data.K, -self.batch_data.K], op="max")
        if int(ks[0]) != -int(ks[1]):
            raise RuntimeError("ranks disagree on the number of nonants per scenario")
        self.nonant_length = self.batch_data.K

    # ------------------------------------------------------------- helpers
    @property
    def local_scenarios(self):
        if not hasattr(self, "_views"):
            self._views = {nm: ScenarioView(self, i) for i, nm in enumerate(self.local_scenario_names)}
        return self._views

    @property
    def local_subproblems(self):
        """phbase.py:1273-1302: the scenarios, or with bundles the bundles
        (name, scen_list, _mpisppy_probability)."""
        if not self.bundling:
            return self.local_scenarios
        if not hasattr(self, "_bundle_views"):
            from .bundles import BundleView
            bl = self.bundle_layout
            mine = self.names_in_bundles[self.cylinder_rank]
            self._bundle_views = {nm: BundleView(nm, mine[b], bl.P[b])
                                  for b, nm in enumerate(bl.names)}
        return self._bundle_views

    @property
    def spcomm(self):
        return self._spcomm

    @spcomm.setter
    def spcomm(self, value):
        if self._spcomm is None:
            self._spcomm = value
        else:
            raise RuntimeError("SPBase.spcomm should only be set once")

    def _options_check(self, required_options, given_options):
        missing = [o for o in required_options if o not in given_options]
        if missing:
            raise ValueError(f"Missing the following required options: {', '.join(missing)}")

    def nonant_names(self):
        d = self.batch_data
        if d.var_names is None:
            return [f"x[{j}]" for j in d.nonant_cols]
        return [d.var_names[j] for j in d.nonant_cols]
