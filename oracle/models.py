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


# ------------------------------------------------------------------- uc -----
# paperruns/larger_uc/ReferenceModel_OK.py (the egret-free, Pyomo-only unit
# commitment model; uc_funcs.py builds egret's "tight" model instead), its
# LP relaxation (binaries in [0, 1]), restated from the model's rules on the
# WECC-240 data of paperruns/larger_uc (tools/make_uc_data.py):
# regulation_services = reserve_services = False, storage_services = True
# with no storage units, one bus, no lines, WIND nondispatchable.
# The reference states PiecewiseProductionCostsConstr once per piece with
# the same body (ReferenceModel_OK.py:1454-1458); the rows are identical, so
# the restatement keeps one per (g, t): same feasible set and objective.
_UC_JSON = None


def _uc_json():
    global _UC_JSON
    if _UC_JSON is None:
        import json
        import os
        here = os.path.dirname(os.path.abspath(__file__))
        path = os.path.join(here, "..", "mpi-sppy_amd", "mpisppy_amd", "examples", "data", "uc_wecc240.json")
        with open(path) as f:
            _UC_JSON = json.load(f)
    return _UC_JSON


def _uc_piecewise(pts, vals, pmin, pmax):
    """ReferenceModel_OK.py:530-585 (points/values are ordered Pyomo Sets:
    duplicates dropped; sorted; min / max output added; clipped; values cut
    or extended by +1, +2, ...)."""
    def uniq(v):
        out = []
        for a in v:
            if a not in out:
                out.append(a)
        return out
    p = sorted(uniq(pts))
    v = sorted(uniq(vals))
    if pmin not in p:
        p.insert(0, pmin)
    if pmax not in p:
        p.append(pmax)
    p = [a for a in p if pmin <= a <= pmax]
    if len(p) < len(v):
        v = v[:len(p)]
    i = 1
    while len(p) > len(v):
        v.append(v[-1] + i)
        i += 1
    return p, v


def uc(scenario_name, scenario_set="1000scenarios_wind"):
    """One UC scenario's LP relaxation (ScenarioN -> NodeN's wind)."""
    d = _uc_json()
    snum = extract_num(scenario_name)
    T = int(d["NumTimePeriods"])
    TPL = float(d["TimePeriodLength"])
    gens = list(d["ThermalGenerators"])
    wind_lo = np.asarray(d["scenario_sets"][scenario_set]["wind_min"][snum - 1])
    wind_hi = np.asarray(d["scenario_sets"][scenario_set]["wind_max"][snum - 1])
    cols = {}          # name -> index
    lo, hi, cost = [], [], []

    def var(name, l_, u_, c_=0.0):
        cols[name] = len(lo)
        lo.append(l_)
        hi.append(u_)
        cost.append(c_)
        return cols[name]

    rows_r, rows_c, rows_v, rl, ru = [], [], [], [], []

    def row(terms, l_, u_):
        r = len(rl)
        acc = {}
        for j, a in terms:
            acc[j] = acc.get(j, 0.0) + a
        for j, a in acc.items():
            if a != 0.0:
                rows_r.append(r)
                rows_c.append(j)
                rows_v.append(a)
        rl.append(l_)
        ru.append(u_)

    INF = np.inf
    on, st, sp_, pg, mp = {}, {}, {}, {}, {}
    pc, suc, sdc, si, pp = {}, {}, {}, {}, {}
    par = {}
    for g in gens:
        t_ = d["gen_table"][g]
        pmin, pmax = t_["MinimumPowerOutput"], t_["MaximumPowerOutput"]
        fuel = t_["FuelCost"]
        pts, vals = _uc_piecewise(d["piecewise_points"][g], d["piecewise_values"][g], pmin, pmax)
        minprod = vals[0] * fuel if len(pts) > 1 else 0.0
        pwp = [a - pmin for a in pts]
        pwv = [b - minprod / fuel for b in vals]
        t0 = t_["UnitOnT0State"]
        u0 = 1 if t0 >= 1 else 0
        mu = min(int(round(t_["MinimumUpTime"] / TPL)), T)
        md = min(int(round(t_["MinimumDownTime"] / TPL)), T)
        on_init = 0 if not u0 else int(min(T, round(max(0, t_["MinimumUpTime"] - t0) / TPL)))
        off_init = 0 if u0 else int(min(T, round(max(0, t_["MinimumDownTime"] + t0) / TPL)))
        lags = list(d["startup_lags"][g])
        scost = list(d["startup_costs"][g])
        vstp = list(range(1, T + 1)) + ([] if t0 >= 0 else [1 + int(t0)])
        pairs = [(tp, tt) for tp in vstp for tt in range(1, T + 1) if lags[0] <= tt - tp < lags[-1]]
        par[g] = dict(pmin=pmin, pmax=pmax, fuel=fuel, pwp=pwp, pwv=pwv, minprod=minprod, u0=u0, mu=mu,
                      md=md, on_init=on_init, off_init=off_init, lags=lags, scost=scost, vstp=vstp,
                      pairs=pairs, pg0=t_["PowerGeneratedT0"],
                      rup=min(t_["NominalRampUpLimit"] * TPL, pmax),
                      rdn=min(t_["NominalRampDownLimit"] * TPL, pmax),
                      sul=min(t_["StartupRampLimit"], pmax), sdl=min(t_["ShutdownRampLimit"], pmax),
                      mut=int(t_["MinimumUpTime"]))
        for t in range(1, T + 1):
            on[g, t] = var(f"UnitOn[{g},{t}]", 0.0, 1.0, minprod * TPL)
            st[g, t] = var(f"UnitStart[{g},{t}]", 0.0, 1.0)
            sp_[g, t] = var(f"UnitStop[{g},{t}]", 0.0, 1.0)
            pg[g, t] = var(f"PowerGeneratedAboveMinimum[{g},{t}]", 0.0, pmax - pmin)
            mp[g, t] = var(f"MaximumPowerAvailableAboveMinimum[{g},{t}]", 0.0, pmax - pmin)
            pc[g, t] = var(f"ProductionCost[{g},{t}]", 0.0, INF, 1.0)
            suc[g, t] = var(f"StartupCost[{g},{t}]", 0.0, INF, 1.0)
            sdc[g, t] = var(f"ShutdownCost[{g},{t}]", 0.0, INF, 1.0)
            for i in range(len(pwp) - 1):
                pp[g, t, i] = var(f"PiecewiseProduction[{g},{t},{i}]", 0.0, pwp[i + 1] - pwp[i])
        for (tp, tt) in pairs:
            si[g, tp, tt] = var(f"StartupIndicator[{g},{tp},{tt}]", 0.0, 1.0)
    nd = {t: var(f"NondispatchablePowerUsed[WIND,{t}]", wind_lo[t - 1], wind_hi[t - 1]) for t in range(1, T + 1)}
    ang = {t: var(f"Angle[SingleBus,{t}]", -3.14159265, 3.14159265) for t in range(1, T + 1)}
    tpc = {t: var(f"TotalProductionCost[{t}]", 0.0, INF) for t in range(1, T + 1)}
    tnl = {t: var(f"TotalNoLoadCost[{t}]", 0.0, INF) for t in range(1, T + 1)}
    lgm = {t: var(f"LoadGenerateMismatch[SingleBus,{t}]", -INF, INF) for t in range(1, T + 1)}
    pos = {t: var(f"posLoadGenerateMismatch[SingleBus,{t}]", 0.0, INF, d["LoadMismatchPenalty"])
           for t in range(1, T + 1)}
    neg = {t: var(f"negLoadGenerateMismatch[SingleBus,{t}]", 0.0, INF, d["LoadMismatchPenalty"])
           for t in range(1, T + 1)}
    rsf = {t: var(f"ReserveShortfall[{t}]", 0.0, INF, 1e5) for t in range(1, T + 1)}
    demand, reserve = d["demand"], d["reserve"]
    # system rows
    row([(pos[t], 1.0) for t in range(1, T + 1)], 0.0, INF)
    row([(neg[t], 1.0) for t in range(1, T + 1)], 0.0, INF)
    for t in range(1, T + 1):
        row([(ang[t], 1.0)], 0.0, 0.0)
        terms = [(nd[t], 1.0), (lgm[t], 1.0)]
        for g in gens:
            terms += [(pg[g, t], 1.0), (on[g, t], par[g]["pmin"])]
        row(terms, demand[t - 1], demand[t - 1])
        row([(pos[t], 1.0), (neg[t], -1.0), (lgm[t], -1.0)], 0.0, 0.0)
        row([(rsf[t], 1.0)], -INF, reserve[t - 1])
        terms = [(nd[t], 1.0), (lgm[t], 1.0), (rsf[t], 1.0)]
        for g in gens:
            terms += [(mp[g, t], 1.0), (on[g, t], par[g]["pmin"])]
        row(terms, demand[t - 1] + reserve[t - 1], INF)
        row([(tpc[t], 1.0)] + [(pc[g, t], -1.0) for g in gens], 0.0, 0.0)
        row([(tnl[t], 1.0)] + [(on[g, t], -par[g]["minprod"]) for g in gens], 0.0, 0.0)
    for g in gens:
        p = par[g]
        span = p["pmax"] - p["pmin"]
        for t in range(1, T + 1):
            row([(pg[g, t], 1.0), (mp[g, t], -1.0)], -INF, 0.0)                      # PartB
            last = t == T
            if p["mut"] == 1:
                row([(mp[g, t], 1.0), (on[g, t], -span), (st[g, t], p["pmax"] - p["sul"])], -INF, 0.0)
                if last:
                    row([(mp[g, t], 1.0), (on[g, t], -span)], -INF, 0.0)
                else:
                    row([(mp[g, t], 1.0), (on[g, t], -span), (sp_[g, t + 1], p["pmax"] - p["sdl"])], -INF, 0.0)
            else:
                terms = [(mp[g, t], 1.0), (on[g, t], -span), (st[g, t], p["pmax"] - p["sul"])]
                if not last:
                    terms.append((sp_[g, t + 1], p["pmax"] - p["sdl"]))
                row(terms, -INF, 0.0)
            if t == 1:                                                              # ramp up / down
                row([(mp[g, 1], 1.0)], -INF, (p["pg0"] - p["pmin"]) * p["u0"] + p["rup"])
                row([(pg[g, 1], -1.0)], -INF, p["rdn"] - (p["pg0"] - p["pmin"]) * p["u0"])
            else:
                row([(mp[g, t], 1.0), (pg[g, t - 1], -1.0)], -INF, p["rup"])
                row([(pg[g, t - 1], 1.0), (pg[g, t], -1.0)], -INF, p["rdn"])
            npc = len(p["pwp"]) - 1
            row([(pp[g, t, i], 1.0) for i in range(npc)] + [(pg[g, t], -1.0)], 0.0, 0.0)
            for i in range(npc):
                row([(pp[g, t, i], 1.0), (on[g, t], -(p["pwp"][i + 1] - p["pwp"][i]))], -INF, 0.0)
            if npc > 0:
                terms = [(pc[g, t], 1.0)]
                for i in range(npc):
                    slope = (TPL * p["pwv"][i + 1] * p["fuel"] - TPL * p["pwv"][i] * p["fuel"]) \
                        / (p["pwp"][i + 1] - p["pwp"][i])
                    terms.append((pp[g, t, i], -slope))
                row(terms, 0.0, 0.0)
            # startup / shutdown matching and costs
            row([(si[g, tp, tt], 1.0) for (tp, tt) in p["pairs"] if tt == t] + [(st[g, t], -1.0)], -INF, 0.0)
            terms = [(suc[g, t], 1.0), (st[g, t], -p["scost"][-1])]
            for s in range(1, len(p["lags"])):
                coef = p["scost"][s - 1] - p["scost"][-1]
                for tp in p["vstp"]:
                    if p["lags"][s - 1] <= t - tp < p["lags"][s]:
                        terms.append((si[g, tp, t], -coef))
            row(terms, 0.0, 0.0)
            row([(sdc[g, t], 1.0)], 0.0, 0.0)                                      # ShutdownFixedCost = 0
            if t >= p["mu"]:
                row([(st[g, i], 1.0) for i in range(max(1, t - p["mu"] + 1), t + 1)] + [(on[g, t], -1.0)],
                    -INF, 0.0)
            if t >= p["md"]:
                row([(sp_[g, i], 1.0) for i in range(max(1, t - p["md"] + 1), t + 1)] + [(on[g, t], 1.0)],
                    -INF, 1.0)
            if t == 1:
                row([(on[g, 1], 1.0), (st[g, 1], -1.0), (sp_[g, 1], 1.0)], p["u0"], p["u0"])
            else:
                row([(on[g, t], 1.0), (on[g, t - 1], -1.0), (st[g, t], -1.0), (sp_[g, t], 1.0)], 0.0, 0.0)
        for tp in p["vstp"]:                                                        # ShutdownMatch
            terms = [(si[g, a, b], 1.0) for (a, b) in p["pairs"] if a == tp]
            if tp < 1:
                if terms:
                    row(terms, -INF, 1.0)
            else:
                row(terms + [(sp_[g, tp], -1.0)], -INF, 0.0)
        if p["on_init"] > 0:
            row([(on[g, t], 1.0) for t in range(1, T + 1) if t <= p["on_init"]], p["on_init"], p["on_init"])
        if p["off_init"] > 0:
            row([(on[g, t], 1.0) for t in range(1, T + 1) if t <= p["off_init"]], 0.0, 0.0)
    n = len(lo)
    A = sp.csr_matrix((rows_v, (rows_r, rows_c)), shape=(len(rl), n))
    names = [None] * n
    for k, j in cols.items():
        names[j] = k
    nonant = [on[g, t] for (g, t) in sorted(on)]     # sorted keys (scenario_tree.py:36)
    return OScen(scenario_name, names, np.asarray(cost), A, np.asarray(rl), np.asarray(ru),
                 np.asarray(lo), np.asarray(hi), [("ROOT", 1.0, nonant)])
