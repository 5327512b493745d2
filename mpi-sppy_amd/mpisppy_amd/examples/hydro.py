"""3-stage hydro (``examples/hydro/hydro.py`` + ``PySP/scenariodata/Scen*.dat``).

The .dat data differ across Scen1..9 only in A[2] (by (snum-1)//3) and A[3]
(by (snum-1)%3); the remaining parameters are common (Scen1.dat).
"""
from ..model import LinearModel
from .. import scenario_tree
from ..utils import sputils

D = {1: 90.0, 2: 160.0, 3: 110.0}
U = {1: 0.6048, 2: 0.6048, 3: 1.2096}
DURACION = {1: 168.0, 2: 168.0, 3: 336.0}
A2 = [10.0, 50.0, 90.0]
A3 = [40.0, 50.0, 60.0]
betaGt, betaGh, betaDns = 1.0, 0.0, 10.0
PgtMin, PgtMax, PghMin, PghMax, VMin, VMax = 0.0, 100.0, 0.0, 100.0, 0.0, 100.0
V0, T = 60.48, 8760.0


def build(snum):
    A = {1: 50.0, 2: A2[(snum - 1) // 3], 3: A3[(snum - 1) % 3]}
    m = LinearModel(f"Scen{snum}")
    etap = [1, 2, 3]
    m.add_var("Pgt", etap, lb=PgtMin, ub=PgtMax)
    m.add_var("Pgh", etap, lb=PghMin, ub=PghMax)
    m.add_var("PDns", etap, lb=0.0, ub=lambda t: D[t])
    m.add_var("Vol", etap, lb=VMin, ub=VMax)
    m.add_var("sl", None, lb=0.0)
    m.add_var("StageCost", etap)
    r = {t: (1 / 1.1) ** (DURACION[t] / T) for t in etap}          # hydro.py:96-99
    for t in etap:                                                  # hydro.py:104-115
        rhs = r[t] * (betaGt * m.Pgt[t] + betaGh * m.Pgh[t] + betaDns * m.PDns[t])
        if t == 3:
            rhs = rhs + m.sl
        m.add_constraint(f"StageCostConstraint[{t}]", m.StageCost[t] == rhs)
    for t in etap:                                                  # hydro.py:122-124
        m.add_constraint(f"demand[{t}]", m.Pgt[t] + m.Pgh[t] + m.PDns[t] - D[t] == 0.0)
    for t in etap:                                                  # hydro.py:127-132
        prev = V0 if t == 1 else m.Vol[t - 1]
        m.add_constraint(f"conserv[{t}]", m.Vol[t] - prev <= U[t] * (A[t] - m.Pgh[t]))
    m.add_constraint("fcfe", m.sl >= 4166.67 * (V0 - m.Vol[3]))    # hydro.py:135-137
    m.set_objective(m.StageCost[1] + m.StageCost[2] + m.StageCost[3], "min")
    return m


def MakeNodesforScen(model, BFs, scennum):
    """hydro.py:181-210."""
    ndn = "ROOT_" + str((scennum - 1) // BFs[0])
    return [
        scenario_tree.ScenarioNode("ROOT", 1.0, 1, model.StageCost[1], None,
                                   [model.Pgt[1], model.Pgh[1], model.PDns[1], model.Vol[1]], model),
        scenario_tree.ScenarioNode(ndn, 1.0 / BFs[0], 2, model.StageCost[2], None,
                                   [model.Pgt[2], model.Pgh[2], model.PDns[2], model.Vol[2]], model,
                                   parent_name="ROOT"),
    ]


def scenario_creator(scenario_name, branching_factors=None, data_path=None):
    if branching_factors is None:
        raise ValueError("Hydro scenario_creator requires branching_factors")
    snum = sputils.extract_num(scenario_name)
    inst = build(snum)
    inst._mpisppy_node_list = MakeNodesforScen(inst, branching_factors, snum)
    return inst


def scenario_denouement(rank, scenario_name, scenario):
    pass


def all_names_and_nodes(BFs=(3, 3)):
    names = [f"Scen{i + 1}" for i in range(BFs[0] * BFs[1])]
    nodes = ["ROOT"] + [f"ROOT_{b}" for b in range(BFs[0])]
    return names, nodes
