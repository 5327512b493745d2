"""Oracle restatement of the reference's scenario generators (TEST INFRASTRUCTURE).

Each generator returns an :class:`OScen` -- a plain sparse LP in the
reference's *own* sense (min or max) plus the scenario-tree node list that
``ScenarioNode``/``build_vardatalist`` would build for it
(``mpisppy/scenario_tree.py:10-38``: nonant vardatas of an indexed Var are
taken in ``sorted(v.keys())`` order).

This module is deliberately written independently of the product's model
builder (``mpi-sppy_amd/mpisppy_amd/examples``); tests check both agree.
"""
import re
import numpy as np
import scipy.sparse as sp


class OScen:
    """One scenario LP:  opt c.x + const  s.t. rl <= A x <= ru, l <= x <= u."""

    def __init__(self, name, var_names, c, A, rl, ru, l, u, nodes,
                 prob=None, sense="min", const=0.0):
        self.name = name
        self.var_names = list(var_names)
        self.c = np.asarray(c, dtype=np.float64)
        self.A = sp.csr_matrix(A, dtype=np.float64)
        self.rl = np.asarray(rl, dtype=np.float64)
        self.ru = np.asarray(ru, dtype=np.float64)
        self.l = np.asarray(l, dtype=np.float64)
        self.u = np.asarray(u, dtype=np.float64)
        # nodes: list of (node_name, cond_prob, [var indices in nonant order])
        self.nodes = nodes
        self.prob = prob
        self.sense = sense
        self.const = float(const)

    @property
    def nonant_idx(self):
        out = []
        for _, _, idx in self.nodes:
            out.extend(idx)
        return np.asarray(out, dtype=np.int64)


def extract_num(s):
    """``mpisppy/utils/sputils.py:414-423``: trailing integer of a name."""
    return int(re.search(r"(\d+)$", s).group(1))


# ---------------------------------------------------------------- farmer ----
# examples/farmer/farmer.py:84-223 (scalable farmer, crops_multiplier)
_F_BASE = ["WHEAT", "CORN", "SUGAR_BEETS"]
_F_PRICE_QUOTA = {"WHEAT": 100000.0, "CORN": 100000.0, "SUGAR_BEETS": 6000.0}
_F_SUB_PRICE = {"WHEAT": 170.0, "CORN": 150.0, "SUGAR_BEETS": 36.0}
_F_SUPER_PRICE = {"WHEAT": 0.0, "CORN": 0.0, "SUGAR_BEETS": 10.0}
_F_CATTLE = {"WHEAT": 200.0, "CORN": 240.0, "SUGAR_BEETS": 0.0}
_F_PURCHASE = {"WHEAT": 238.0, "CORN": 210.0, "SUGAR_BEETS": 100000.0}
_F_PLANT = {"WHEAT": 150.0, "CORN": 230.0, "SUGAR_BEETS": 260.0}
_F_YIELD = {  # farmer.py:142-148
    "BelowAverageScenario": {"WHEAT": 2.0, "CORN": 2.4, "SUGAR_BEETS": 16.0},
    "AverageScenario": {"WHEAT": 2.5, "CORN": 3.0, "SUGAR_BEETS": 20.0},
    "AboveAverageScenario": {"WHEAT": 3.0, "CORN": 3.6, "SUGAR_BEETS": 24.0},
}


def farmer_yields(scennum, crops_multiplier=1):
    """Yield per crop in CROPS order (farmer.py:44-54,150-156).

    CROPS = [WHEAT0, CORN0, SUGAR_BEETS0, WHEAT1, ...] (farmer.py:98-104);
    the stream is re-seeded with the scenario number (farmer.py:54) and one
    ``rand()`` is drawn per crop, in CROPS order, when groupnum != 0.
    """
    basenames = ["BelowAverageScenario", "AverageScenario", "AboveAverageScenario"]
    base = basenames[scennum % 3]
    groupnum = scennum // 3
    rs = np.random.RandomState(scennum)
    ys = []
    for i in range(crops_multiplier):
        for crop in _F_BASE:
            y = _F_YIELD[base][crop]
            if groupnum != 0:
                y = y + rs.rand()
            ys.append(y)
    return ys


def farmer(scenario_name, crops_multiplier=1, sense="min", num_scens=None):
    """Scalable farmer scenario (farmer.py:24-82)."""
    c = crops_multiplier
    scennum = extract_num(scenario_name)
    crops = [f"{b}{i}" for i in range(c) for b in _F_BASE]
    ncr = len(crops)
    yields = farmer_yields(scennum, c)
    # variable blocks in declaration order (farmer.py:167-177)
    DA = lambda k: k
    QSUB = lambda k: ncr + k
    QSUP = lambda k: 2 * ncr + k
    QP = lambda k: 3 * ncr + k
    n = 4 * ncr
    names = ([f"DevotedAcreage[{x}]" for x in crops]
             + [f"QuantitySubQuotaSold[{x}]" for x in crops]
             + [f"QuantitySuperQuotaSold[{x}]" for x in crops]
             + [f"QuantityPurchased[{x}]" for x in crops])
    base = lambda x: x.rstrip("0123456789")
    cost = np.zeros(n)
    for k, x in enumerate(crops):
        b = base(x)
        cost[DA(k)] = _F_PLANT[b]          # FirstStageCost  (farmer.py:205-207)
        cost[QP(k)] = _F_PURCHASE[b]       # SecondStageCost (farmer.py:209-214)
        cost[QSUB(k)] = -_F_SUB_PRICE[b]
        cost[QSUP(k)] = -_F_SUPER_PRICE[b]
    if sense == "max":                     # farmer.py:216-221
        cost = -cost
    rows, cols, vals, rl, ru = [], [], [], [], []
    r = 0
    # ConstrainTotalAcreage  sum DA <= 500c   (farmer.py:183-186)
    for k in range(ncr):
        rows.append(r); cols.append(DA(k)); vals.append(1.0)
    rl.append(-np.inf); ru.append(500.0 * c); r += 1
    # EnforceCattleFeedRequirement  (farmer.py:188-191)
    for k, x in enumerate(crops):
        for j, v in ((DA(k), yields[k]), (QP(k), 1.0), (QSUB(k), -1.0), (QSUP(k), -1.0)):
            rows.append(r); cols.append(j); vals.append(v)
        rl.append(_F_CATTLE[base(x)]); ru.append(np.inf); r += 1
    # LimitAmountSold  (farmer.py:193-196)
    for k, x in enumerate(crops):
        for j, v in ((QSUB(k), 1.0), (QSUP(k), 1.0), (DA(k), -yields[k])):
            rows.append(r); cols.append(j); vals.append(v)
        rl.append(-np.inf); ru.append(0.0); r += 1
    # EnforceQuotas  0 <= QSUB <= PriceQuota  (farmer.py:198-201)
    for k, x in enumerate(crops):
        rows.append(r); cols.append(QSUB(k)); vals.append(1.0)
        rl.append(0.0); ru.append(_F_PRICE_QUOTA[base(x)]); r += 1
    A = sp.csr_matrix((vals, (rows, cols)), shape=(r, n))
    l = np.zeros(n)
    u = np.full(n, np.inf)
    u[:ncr] = 500.0 * c                   # farmer.py:172-173
    # nonants: DevotedAcreage in sorted key order (scenario_tree.py:36)
    order = sorted(range(ncr), key=lambda k: crops[k])
    nodes = [("ROOT", 1.0, [DA(k) for k in order])]
    prob = None if num_scens is None else 1.0 / num_scens
    return OScen(scenario_name, names, cost, A, rl, ru, l, u, nodes,
                 prob=prob, sense=sense)


# ------------------------------------------------------- doc textbook farmer
# doc/src/examples.rst:50-92 (build_model) and :155-175 (scenario_creator)
def doc_farmer(scenario_name):
    ylds = {"good": [3, 3.6, 24], "average": [2.5, 3, 20], "bad": [2, 2.4, 16]}[scenario_name]
    # vars: X[WHEAT,CORN,BEETS], Y[WHEAT,CORN], W[WHEAT,CORN,BEETS_FAVORABLE,BEETS_UNFAVORABLE]
    names = ["X[WHEAT]", "X[CORN]", "X[BEETS]", "Y[WHEAT]", "Y[CORN]",
             "W[WHEAT]", "W[CORN]", "W[BEETS_FAVORABLE]", "W[BEETS_UNFAVORABLE]"]
    c = np.array([150, 230, 260, 238, 210, -170, -150, -36, -10], dtype=float)
    A = np.zeros((4, 9))
    A[0, 0:3] = 1.0
    A[1, 0] = ylds[0]; A[1, 3] = 1; A[1, 5] = -1
    A[2, 1] = ylds[1]; A[2, 4] = 1; A[2, 6] = -1
    A[3, 2] = ylds[2]; A[3, 7] = -1; A[3, 8] = -1
    rl = np.array([-np.inf, 200, 240, 0.0])
    ru = np.array([500, np.inf, np.inf, np.inf])
    l = np.zeros(9)
    u = np.full(9, np.inf)
    u[7] = 6000.0
    # attach_root_node(model, PLANTING_COST, [model.X]): sorted keys BEETS, CORN, WHEAT
    nodes = [("ROOT", 1.0, [2, 1, 0])]
    return OScen(scenario_name, names, c, sp.csr_matrix(A), rl, ru, l, u, nodes,
                 prob=1.0 / 3)


# ----------------------------------------------------------------- hydro ----
# examples/hydro/hydro.py:33-145 with PySP/scenariodata/Scen{1..9}.dat
_H_D = [90.0, 160.0, 110.0]
_H_U = [0.6048, 0.6048, 1.2096]
_H_DUR = [168.0, 168.0, 336.0]
_H_A2 = [10.0, 50.0, 90.0]     # Scen{1-3,4-6,7-9}.dat  "param A" row 2
_H_A3 = [40.0, 50.0, 60.0]     # Scen{1,4,7},{2,5,8},{3,6,9}.dat row 3


def hydro(scenario_name, branching_factors=(3, 3)):
    snum = extract_num(scenario_name)
    A = [50.0, _H_A2[(snum - 1) // 3], _H_A3[(snum - 1) % 3]]
    T, V0 = 8760.0, 60.48
    betaGt, betaGh, betaDns = 1.0, 0.0, 10.0
    r = [(1 / 1.1) ** (_H_DUR[t] / T) for t in range(3)]   # hydro.py:96-99
    # var layout: Pgt[1..3], Pgh[1..3], PDns[1..3], Vol[1..3], sl, StageCost[1..3]
    Pgt = lambda t: t; Pgh = lambda t: 3 + t; PDns = lambda t: 6 + t
    Vol = lambda t: 9 + t; SL = 12; SC = lambda t: 13 + t
    n = 16
    names = ([f"Pgt[{t+1}]" for t in range(3)] + [f"Pgh[{t+1}]" for t in range(3)]
             + [f"PDns[{t+1}]" for t in range(3)] + [f"Vol[{t+1}]" for t in range(3)]
             + ["sl"] + [f"StageCost[{t+1}]" for t in range(3)])
    Am = np.zeros((10, n)); rl = np.zeros(10); ru = np.zeros(10)
    i = 0
    for t in range(3):   # StageCostConstraint (hydro.py:104-115)
        Am[i, SC(t)] = 1.0
        Am[i, Pgt(t)] = -r[t] * betaGt
        Am[i, Pgh(t)] = -r[t] * betaGh
        Am[i, PDns(t)] = -r[t] * betaDns
        if t == 2:
            Am[i, SL] = -1.0
        rl[i] = ru[i] = 0.0; i += 1
    for t in range(3):   # demand (hydro.py:122-124)
        Am[i, Pgt(t)] = Am[i, Pgh(t)] = Am[i, PDns(t)] = 1.0
        rl[i] = ru[i] = _H_D[t]; i += 1
    for t in range(3):   # conserv (hydro.py:127-132)
        Am[i, Vol(t)] = 1.0
        if t > 0:
            Am[i, Vol(t - 1)] = -1.0
        Am[i, Pgh(t)] = _H_U[t]
        rl[i] = -np.inf
        ru[i] = _H_U[t] * A[t] + (V0 if t == 0 else 0.0); i += 1
    # fcfe  sl >= 4166.67*(V0 - Vol[3])  (hydro.py:135-137)
    Am[i, SL] = 1.0; Am[i, Vol(2)] = 4166.67
    rl[i] = 4166.67 * V0; ru[i] = np.inf; i += 1
    l = np.zeros(n); u = np.zeros(n)
    for t in range(3):   # hydro.py:67-88
        u[Pgt(t)] = 100.0; u[Pgh(t)] = 100.0; u[PDns(t)] = _H_D[t]; u[Vol(t)] = 100.0
    u[SL] = np.inf
    for t in range(3):
        l[SC(t)] = -np.inf; u[SC(t)] = np.inf
    c = np.zeros(n)
    for t in range(3):
        c[SC(t)] = 1.0   # hydro.py:149-151
    bf = branching_factors
    ndn = "ROOT_" + str((snum - 1) // bf[0])      # hydro.py:189
    nodes = [("ROOT", 1.0, [Pgt(0), Pgh(0), PDns(0), Vol(0)]),
             (ndn, 1.0 / bf[0], [Pgt(1), Pgh(1), PDns(1), Vol(1)])]
    return OScen(scenario_name, names, c, sp.csr_matrix(Am), rl, ru, l, u, nodes)


# ------------------------------------------------------------------ sslp ----
# examples/sslp/model/ReferenceModel.py:22-94 (LP relaxation: binaries in
# [0, 1]), scenario_creator sslp.py:17-33.  Instance data: the reference's
# data/<inst>/scenariodata/Scenario*.dat, converted to JSON by
# tools/make_sslp_data.py (mpi-sppy_amd/mpisppy_amd/examples/data/sslp.json).
_SSLP_JSON = None


def _sslp_json():
    global _SSLP_JSON
    if _SSLP_JSON is None:
        import json
        import os
        here = os.path.dirname(os.path.abspath(__file__))
        path = os.path.join(here, "..", "mpi-sppy_amd", "mpisppy_amd", "examples", "data", "sslp.json")
        with open(path) as f:
            _SSLP_JSON = json.load(f)
    return _SSLP_JSON


def sslp(scenario_name, instance="sslp_15_45_5"):
    d = _sslp_json()
    snum = extract_num(scenario_name)
    m_ = re.fullmatch(r"sslp_(\d+)_(\d+)_synthetic", instance)
    if m_:
        size = d["sizes"][f"{m_.group(1)}_{m_.group(2)}"]
        present = (np.random.RandomState(1134 + snum).rand(size["NumClients"]) < 0.5) * 1.0
    else:
        inst = d["instances"][instance]
        size = d["sizes"][inst["size"]]
        present = np.asarray(inst["ClientPresent"][snum - 1], dtype=np.float64)
    J, I = size["NumServers"], size["NumClients"]
    dem = np.asarray(size["Demand"])          # [I][J]
    rev = np.asarray(size["Revenue"])         # [I][J]
    # variables: FacilityOpen[J], Allocation[I][J] (client major), Dummy[J]
    n = J + I * J + J
    yo = np.arange(J)
    xa = (J + np.arange(I * J)).reshape(I, J)
    du = J + I * J + np.arange(J)
    A = np.zeros((J + I, n))
    rl = np.zeros(J + I)
    ru = np.zeros(J + I)
    for j in range(J):          # demand_constraint_rule: sum_i d x - u_j - cap y_j <= 0
        A[j, xa[:, j]] = dem[:, j]
        A[j, du[j]] = -1.0
        A[j, yo[j]] = -size["Capacity"]
        rl[j], ru[j] = -np.inf, 0.0
    for i in range(I):          # client_rule: sum_j x_ij = present_i
        A[J + i, xa[i, :]] = 1.0
        rl[J + i] = ru[J + i] = present[i]
    c = np.zeros(n)
    c[yo] = size["FixedCost"]
    c[du] = 1000.0              # Penalty default
    c[xa] = -rev
    l = np.zeros(n)
    u = np.ones(n)
    u[du] = np.inf
    names = ([f"FacilityOpen[{j + 1}]" for j in range(J)]
             + [f"Allocation[{(i + 1, j + 1)}]" for i in range(I) for j in range(J)]
             + [f"Dummy[{j + 1}]" for j in range(J)])
    nodes = [("ROOT", 1.0, list(yo))]
    return OScen(scenario_name, names, c, sp.csr_matrix(A), rl, ru, l, u, nodes)
