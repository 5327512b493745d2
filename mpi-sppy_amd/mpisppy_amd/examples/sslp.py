"""SSLP LP relaxation (``examples/sslp/sslp.py`` + ``model/ReferenceModel.py``).

Stochastic server location: FacilityOpen[j] (first stage, the nonants),
Allocation[i,j] and Dummy[j] (second stage); the binaries are relaxed to
[0, 1] (ReferenceModel.py keeps the commented-out ``bounds=(0,1)`` forms of
the LP relaxation).  Scenarios differ only in
ClientPresent.  The instance data of the reference's ``data/<inst>/
scenariodata/Scenario*.dat`` files are in ``data/sslp.json``
(``tools/make_sslp_data.py``).  ``instance="sslp_<S>_<C>_synthetic"`` gives
any number of scenarios of an S-server / C-client size with ClientPresent ~
Bernoulli(0.5) from ``RandomState(1134 + scennum)`` (1134: the reference's
default ``--seed``, baseparsers.py).
"""
import json
import os
import re

import numpy as np

from ..batch import BatchData, NodeInfo
from ..model import LinearModel
from .. import scenario_tree
from ..utils import sputils

_DATA = None


def _data():
    global _DATA
    if _DATA is None:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "sslp.json")) as f:
            _DATA = json.load(f)
    return _DATA


def _instance_of(data_dir=None, instance=None):
    if instance is None:
        if data_dir is None:
            raise ValueError("kwarg `data_dir` is required for SSLP scenario_creator")
        hit = re.findall(r"(sslp_\d+_\d+_\w+)", str(data_dir))
        if not hit:
            raise ValueError(f"cannot tell the sslp instance from data_dir={data_dir!r}")
        instance = hit[-1]
    return instance


def instance_data(instance, scennum):
    """(size dict, ClientPresent vector) of scenario `scennum` (1-based)."""
    d = _data()
    m = re.fullmatch(r"sslp_(\d+)_(\d+)_synthetic", instance)
    if m:
        size = d["sizes"][f"{m.group(1)}_{m.group(2)}"]
        rng = np.random.RandomState(1134 + scennum)
        return size, (rng.rand(size["NumClients"]) < 0.5).astype(np.float64)
    inst = d["instances"][instance]
    return d["sizes"][inst["size"]], np.asarray(inst["ClientPresent"][scennum - 1], dtype=np.float64)


def build(instance, scennum):
    size, present = instance_data(instance, scennum)
    ns, nc = size["NumServers"], size["NumClients"]
    servers = list(range(1, ns + 1))
    clients = list(range(1, nc + 1))
    dem = size["Demand"]
    rev = size["Revenue"]
    mdl = LinearModel(f"Scenario{scennum}")
    mdl.add_var("FacilityOpen", servers, lb=0.0, ub=1.0)                       # ReferenceModel.py:54
    mdl.add_var("Allocation", [(i, j) for i in clients for j in servers], lb=0.0, ub=1.0)  # :57
    mdl.add_var("Dummy", servers, lb=0.0)                                      # :60
    for j in servers:                                                          # :67-69
        e = -1.0 * mdl.Dummy[j] - size["Capacity"] * mdl.FacilityOpen[j]
        for i in clients:
            if dem[i - 1][j - 1] != 0.0:
                e = e + dem[i - 1][j - 1] * mdl.Allocation[i, j]
        mdl.add_constraint(f"DemandConstraint[{j}]", e <= 0.0)
    for i in clients:                                                          # :71-73
        e = mdl.Allocation[i, 1] * 1.0
        for j in servers[1:]:
            e = e + mdl.Allocation[i, j]
        mdl.add_constraint(f"ClientConstraint[{i}]", e == float(present[i - 1]))
    first = 0.0 * mdl.FacilityOpen[1]
    for j in servers:                                                          # :79-81
        first = first + size["FixedCost"][j - 1] * mdl.FacilityOpen[j]
    second = 0.0 * mdl.Dummy[1]
    for j in servers:                                                          # :83-85
        second = second + 1000.0 * mdl.Dummy[j]
        for i in clients:
            if rev[i - 1][j - 1] != 0.0:
                second = second - rev[i - 1][j - 1] * mdl.Allocation[i, j]
    mdl.add_expression("FirstStageCost", first)
    mdl.add_expression("SecondStageCost", second)
    mdl.set_objective(first + second, "min")                                   # :91-94
    return mdl


def scenario_creator(scenario_name, data_dir=None, instance=None):
    """sslp.py:17-33: one ROOT node with the FacilityOpen nonants."""
    inst = _instance_of(data_dir, instance)
    snum = sputils.extract_num(scenario_name)
    model = build(inst, snum)
    model._mpisppy_node_list = [
        scenario_tree.ScenarioNode("ROOT", 1.0, 1, model.FirstStageCost, None,
                                   [model.FacilityOpen], model)
    ]
    return model


def batch_creator(scenario_names, data_dir=None, instance=None):
    """All scenarios at once as a :class:`BatchData` (the same numbers as
    ``scenario_creator``; columns FacilityOpen[1..ns], Allocation[i,j] (i
    major), Dummy[1..ns]; rows DemandConstraint[1..ns], ClientConstraint[1..nc])."""
    inst = _instance_of(data_dir, instance)
    nums = [sputils.extract_num(nm) for nm in scenario_names]
    size, _ = instance_data(inst, nums[0])
    ns, nc = size["NumServers"], size["NumClients"]
    S = len(scenario_names)
    OPEN = np.arange(ns)
    ALLOC = lambda i, j: ns + i * ns + j          # noqa: E731 (0-based i, j)
    DUMMY = ns + nc * ns + np.arange(ns)
    n = ns + nc * ns + ns
    dem = np.asarray(size["Demand"])
    rev = np.asarray(size["Revenue"])
    row_ptr, col_idx, vals = [0], [], []
    for j in range(ns):
        cols = {int(OPEN[j]): -size["Capacity"], int(DUMMY[j]): -1.0}
        for i in range(nc):
            if dem[i, j] != 0.0:
                cols[ALLOC(i, j)] = dem[i, j]
        for cc in sorted(cols):
            col_idx.append(cc)
            vals.append(cols[cc])
        row_ptr.append(len(col_idx))
    for i in range(nc):
        for j in range(ns):
            col_idx.append(ALLOC(i, j))
            vals.append(1.0)
        row_ptr.append(len(col_idx))
    m_ = ns + nc
    V = np.repeat(np.asarray(vals)[:, None], S, axis=1)
    cvec = np.zeros(n)
    cvec[OPEN] = size["FixedCost"]
    cvec[DUMMY] = 1000.0
    for i in range(nc):
        for j in range(ns):
            cvec[ALLOC(i, j)] = -rev[i, j]
    c = np.repeat(cvec[:, None], S, axis=1)
    l = np.zeros((n, S))
    u = np.ones((n, S))
    u[DUMMY, :] = np.inf
    rl = np.zeros((m_, S))
    ru = np.zeros((m_, S))
    rl[:ns, :] = -np.inf
    for s, sn in enumerate(nums):
        _, present = instance_data(inst, sn)
        rl[ns:, s] = present
        ru[ns:, s] = present
    names = ([f"FacilityOpen[{j + 1}]" for j in range(ns)]
             + [f"Allocation[{(i + 1, j + 1)}]" for i in range(nc) for j in range(ns)]
             + [f"Dummy[{j + 1}]" for j in range(ns)])
    infos = [NodeInfo([("ROOT", 1.0, ns)])] * S
    return BatchData(scenario_names, np.asarray(row_ptr), np.asarray(col_idx), V, c, np.zeros(S),
                     l, u, rl, ru, OPEN.copy(), infos, "min", var_names=names)


scenario_creator.batch_creator = batch_creator


def scenario_denouement(rank, scenario_name, scenario):
    pass


def scenario_names(num):
    """sslp.py:138-140."""
    return [f"Scenario{sn + 1}" for sn in range(num)]
