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
        if "bundles_per_rank" in options and options["bundles_per_rank"]:
            raise NotImplementedError("bundles_per_rank > 0: bundling is not on the batched hot path")
        self.bundling = False
        if "branching_factors" in options:
            self.branching_factors = options["branching_factors"]
        else:
            self.branching_factors = [len(self.all_scenario_names)]
        self._calculate_scenario_ranks()
        self._create_scenarios(scenario_creator_kwargs)
        self._look_and_leap()
        self._compute_unconditional_node_probabilities()
        self._create_node_slots()
        self._verify_nonant_lengths()
        self.is_minimizing = self.batch_data.sense == "min"
        self._spcomm = None

    # ---------------------------------------------------------------- setup
    def _calculate_scenario_ranks(self):
        self._rank_slices, self._scenario_slices = sputils.scen_names_to_ranks(
            self.all_scenario_names, self.n_proc)
        self.local_scenario_indices = self._rank_slices[self.cylinder_rank]
        self.local_scenario_names = [self.all_scenario_names[i] for i in self.local_scenario_indices]
        self.local_begin = self.local_scenario_indices[0]
        self.local_end = self.local_scenario_indices[-1] + 1

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
        return self.local_scenarios

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
