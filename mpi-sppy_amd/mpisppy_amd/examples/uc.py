"""Unit commitment, LP relaxation (BASELINE config 4).

The reference's UC driver (``paperruns/larger_uc/uc_funcs.py:17-46``) builds
egret's tight model, which is not part of the reference.  The reference also
ships the egret-free, Pyomo-only formulation this example restates:
``paperruns/larger_uc/ReferenceModel_OK.py`` (flags at :18-27:
regulation_services = reserve_services = False, storage_services = True),
on the WECC-240 data of ``paperruns/larger_uc/{1000,3}scenarios_wind``
(``RootNode.dat`` + ``NodeN.dat``: the scenarios differ in the wind bounds;
converted to ``data/uc_wecc240.json`` by ``tools/make_uc_data.py``), with the
binaries relaxed to [0, 1].  Scenario ``ScenarioN`` reads ``NodeN``
(uc_funcs.py:27-32).  UnitOn[*,*] are the nonants (uc_funcs.py:71-78),
rho from ``scenario_rhos`` (uc_funcs.py:94-112).

The reference states ``PiecewiseProductionCostsConstr`` once per piece with
the same body (ReferenceModel_OK.py:1454-1458); one row per (g, t) is kept
(identical rows: same feasible set and objective).  No Storage, lines or
must-run units exist in the data, so those rules add no rows.

Parity is unpinned: no reference file holds a UC LP-relaxation value.
"""
import json
import os

import numpy as np

from ..batch import BatchData, NodeInfo, from_models
from ..model import LinearModel
from .. import scenario_tree
from ..utils import sputils

_DATA = None


def _data():
    global _DATA
    if _DATA is None:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "uc_wecc240.json")) as f:
            _DATA = json.load(f)
    return _DATA


def _scenario_set(path=None, scenario_count=None):
    """uc_cylinders.py:61-64: path = '<count>scenarios_wind'."""
    if path is not None:
        base = os.path.basename(os.path.normpath(str(path)))
        if base in _data()["scenario_sets"]:
            return base
    if scenario_count is not None and int(scenario_count) > 50:
        return "1000scenarios_wind"
    return "3scenarios_wind" if scenario_count is not None else "1000scenarios_wind"


def _ordered_set(v):
    out = []
    for a in v:
        if a not in out:
            out.append(a)
    return out


class Params:
    """The model's derived parameters (ReferenceModel_OK.py:340-812)."""

    def __init__(self):
        d = _data()
        self.T = int(d["NumTimePeriods"])
        self.TPL = float(d["TimePeriodLength"])
        self.G = list(d["ThermalGenerators"])
        self.demand = list(d["demand"])
        self.reserve = list(d["reserve"])
        self.penalty = float(d["LoadMismatchPenalty"])
        self.reserve_penalty = 1e5                     # ModeratelyBigPenalty (:117)
        self.g = {}
        T, TPL = self.T, self.TPL
        for g in self.G:
            r = d["gen_table"][g]
            pmin, pmax = r["MinimumPowerOutput"], r["MaximumPowerOutput"]
            # ValidateCostPiecewisePointsAndValues (:530-585)
            pts = sorted(_ordered_set(d["piecewise_points"][g]))
            vals = sorted(_ordered_set(d["piecewise_values"][g]))
            if pmin not in pts:
                pts.insert(0, pmin)
            if pmax not in pts:
                pts.append(pmax)
            pts = [p for p in pts if pmin <= p <= pmax]
            if len(pts) < len(vals):
                vals = vals[:len(pts)]
            k = 1
            while len(pts) > len(vals):
                vals.append(vals[-1] + k)
                k += 1
            fuel = r["FuelCost"]
            minprod = vals[0] * fuel if len(pts) > 1 else 0.0          # :603-611
            t0 = r["UnitOnT0State"]
            u0 = int(t0 >= 1)                                          # :420-423
            q = dict(
                pmin=pmin, pmax=pmax, fuel=fuel, minprod=minprod, t0=t0, u0=u0, pg0=r["PowerGeneratedT0"],
                points=[p - pmin for p in pts],                        # :643-690 ("Absolute")
                values=[v - minprod / fuel for v in vals],
                ramp_up=min(r["NominalRampUpLimit"] * TPL, pmax),      # :357-371
                ramp_dn=min(r["NominalRampDownLimit"] * TPL, pmax),
                su_lim=min(r["StartupRampLimit"], pmax),               # :373-387
                sd_lim=min(r["ShutdownRampLimit"], pmax),
                min_up=int(r["MinimumUpTime"]), min_dn=int(r["MinimumDownTime"]),
                smin_up=min(int(round(r["MinimumUpTime"] / TPL)), T),  # :397-405
                smin_dn=min(int(round(r["MinimumDownTime"] / TPL)), T),
                lags=list(d["startup_lags"][g]), scosts=list(d["startup_costs"][g]))
            q["on_init"] = 0 if not u0 else int(min(T, round(max(0, q["min_up"] - t0) / TPL)))   # :445-452
            q["off_init"] = 0 if u0 else int(min(T, round(max(0, q["min_dn"] + t0) / TPL)))  # :454-461
            # ValidShutdownTimePeriods / ShutdownHotStartupPairs (:1020-1027)
            q["vstp"] = list(range(1, T + 1)) + ([] if t0 >= 0 else [1 + int(t0)])
            q["pairs"] = [(tp, t) for tp in q["vstp"] for t in range(1, T + 1)
                          if q["lags"][0] <= t - tp < q["lags"][-1]]
            self.g[g] = q

    def production_cost(self, g, t, x):
        """production_cost_function (:1431-1432)."""
        q = self.g[g]
        return self.TPL * q["values"][q["points"].index(x)] * q["fuel"]

    def compute_production_costs(self, g, t, avg_power):
        """compute_production_costs_rule (:1470-1488), literally: the
        buckets compare the absolute avg_power with points relative to the
        minimum output."""
        pts = self.g[g]["points"]
        ev = [0.0] * (len(pts) - 1)
        for l in range(len(ev)):
            if avg_power >= pts[l + 1]:
                ev[l] = pts[l + 1] - pts[l]
            elif avg_power < pts[l + 1]:
                ev[l] = avg_power - pts[l]
                break
        return sum((self.production_cost(g, t, pts[l + 1]) - self.production_cost(g, t, pts[l]))
                   / (pts[l + 1] - pts[l]) * ev[l] for l in range(len(ev)))


_PARAMS = None


def params():
    global _PARAMS
    if _PARAMS is None:
        _PARAMS = Params()
    return _PARAMS


def scenario_creator(scenario_name, path=None, scenario_count=None):
    """uc_funcs.scenario_creator (:48-49) on ReferenceModel_OK's rules."""
    P = params()
    d = _data()
    sset = _scenario_set(path, scenario_count)
    snum = sputils.extract_num(scenario_name)
    wlo = d["scenario_sets"][sset]["wind_min"][snum - 1]
    whi = d["scenario_sets"][sset]["wind_max"][snum - 1]
    T = P.T
    TP = range(1, T + 1)
    G = P.G
    gt = [(g, t) for g in G for t in TP]
    m = LinearModel(scenario_name)
    g_ = P.g
    # -- variables (:1010-1151)
    m.add_var("UnitOn", gt, lb=0.0, ub=1.0)
    m.add_var("UnitStart", gt, lb=0.0, ub=1.0)
    m.add_var("UnitStop", gt, lb=0.0, ub=1.0)
    m.add_var("StartupIndicator", [(g, tp, t) for g in G for (tp, t) in g_[g]["pairs"]], lb=0.0, ub=1.0)
    m.add_var("PowerGeneratedAboveMinimum", gt, lb=0.0, ub=lambda k: g_[k[0]]["pmax"] - g_[k[0]]["pmin"])
    m.add_var("NondispatchablePowerUsed", [("WIND", t) for t in TP], lb=lambda k: wlo[k[1] - 1],
              ub=lambda k: whi[k[1] - 1])
    m.add_var("MaximumPowerAvailableAboveMinimum", gt, lb=0.0,
              ub=lambda k: g_[k[0]]["pmax"] - g_[k[0]]["pmin"])
    m.add_var("Angle", [("SingleBus", t) for t in TP], lb=-3.14159265, ub=3.14159265)
    m.add_var("ProductionCost", gt, lb=0.0)
    m.add_var("StartupCost", gt, lb=0.0)
    m.add_var("ShutdownCost", gt, lb=0.0)
    m.add_var("TotalProductionCost", list(TP), lb=0.0)
    m.add_var("TotalNoLoadCost", list(TP), lb=0.0)
    m.add_var("LoadGenerateMismatch", [("SingleBus", t) for t in TP])
    m.add_var("posLoadGenerateMismatch", [("SingleBus", t) for t in TP], lb=0.0)
    m.add_var("negLoadGenerateMismatch", [("SingleBus", t) for t in TP], lb=0.0)
    m.add_var("ReserveShortfall", list(TP), lb=0.0)
    pw = [(g, t, i) for g in G for t in TP for i in range(len(g_[g]["points"]) - 1)]
    m.add_var("PiecewiseProduction", pw, lb=0.0,
              ub=lambda k: g_[k[0]]["points"][k[2] + 1] - g_[k[0]]["points"][k[2]])
    ON, ST, SP = m.UnitOn, m.UnitStart, m.UnitStop
    PG, MP, SI = m.PowerGeneratedAboveMinimum, m.MaximumPowerAvailableAboveMinimum, m.StartupIndicator
    ND, LGM = m.NondispatchablePowerUsed, m.LoadGenerateMismatch
    POS, NEG, RS = m.posLoadGenerateMismatch, m.negLoadGenerateMismatch, m.ReserveShortfall
    PC, SUC, SDC = m.ProductionCost, m.StartupCost, m.ShutdownCost
    PP = m.PiecewiseProduction

    def total(terms):
        e = 0.0
        for v in terms:
            e = e + v
        return e
    # -- constraints, in the model's declaration order
    for t in TP:
        m.add_constraint(f"FixFirstAngle[{t}]", m.Angle["SingleBus", t] == 0.0)
    m.add_constraint("PosLoadGenerateMismatchTolerance[SingleBus]", total(POS["SingleBus", t] for t in TP) >= 0.0)
    m.add_constraint("NegLoadGenerateMismatchTolerance[SingleBus]", total(NEG["SingleBus", t] for t in TP) >= 0.0)
    for t in TP:   # power_balance (:1169-1185)
        m.add_constraint(f"PowerBalance[SingleBus,{t}]",
                         total(PG[g, t] + g_[g]["pmin"] * ON[g, t] for g in G) + ND["WIND", t]
                         + LGM["SingleBus", t] == P.demand[t - 1])
    for t in TP:
        m.add_constraint(f"DefinePosNegLoadGenerateMismatch[SingleBus,{t}]",
                         POS["SingleBus", t] - NEG["SingleBus", t] == LGM["SingleBus", t])
    for t in TP:
        m.add_constraint(f"BoundReserveShortfall[{t}]", RS[t] <= P.reserve[t - 1])
    for t in TP:   # enforce_reserve_requirements_rule (:1204-1222)
        m.add_constraint(f"EnforceReserveRequirements[{t}]",
                         total(MP[g, t] + g_[g]["pmin"] * ON[g, t] for g in G) + ND["WIND", t]
                         + LGM["SingleBus", t] + RS[t] >= P.demand[t - 1] + P.reserve[t - 1])
    for g, t in gt:
        m.add_constraint(f"EnforceGeneratorOutputLimitsPartB[{g},{t}]", PG[g, t] <= MP[g, t])
    for g, t in gt:   # power_limit_from_start (:1283-1289)
        q = g_[g]
        if q["min_up"] != 1:
            continue
        m.add_constraint(f"power_limit_from_start[{g},{t}]",
                         MP[g, t] <= (q["pmax"] - q["pmin"]) * ON[g, t] - (q["pmax"] - q["su_lim"]) * ST[g, t])
    for g, t in gt:   # power_limit_from_stop (:1291-1299)
        q = g_[g]
        if q["min_up"] != 1:
            continue
        if t == T:
            m.add_constraint(f"power_limit_from_stop[{g},{t}]", MP[g, t] <= (q["pmax"] - q["pmin"]) * ON[g, t])
        else:
            m.add_constraint(f"power_limit_from_stop[{g},{t}]",
                             MP[g, t] <= (q["pmax"] - q["pmin"]) * ON[g, t]
                             - (q["pmax"] - q["sd_lim"]) * SP[g, t + 1])
    for g, t in gt:   # power_limit_from_start_stop (:1301-1311)
        q = g_[g]
        if q["min_up"] == 1:
            continue
        e = (q["pmax"] - q["pmin"]) * ON[g, t] - (q["pmax"] - q["su_lim"]) * ST[g, t]
        if t != T:
            e = e - (q["pmax"] - q["sd_lim"]) * SP[g, t + 1]
        m.add_constraint(f"power_limit_from_start_stop[{g},{t}]", MP[g, t] <= e)
    for g, t in gt:   # enforce_max_available_ramp_up_rates_rule (:1321-1330)
        q = g_[g]
        if t == 1:
            m.add_constraint(f"EnforceMaxAvailableRampUpRates[{g},{t}]",
                             MP[g, t] <= (q["pg0"] - q["pmin"]) * q["u0"] + q["ramp_up"])
        else:
            m.add_constraint(f"EnforceMaxAvailableRampUpRates[{g},{t}]", MP[g, t] <= PG[g, t - 1] + q["ramp_up"])
    for g, t in gt:   # enforce_ramp_down_limits_rule (:1336-1347), enforce_t1_ramp_rates
        q = g_[g]
        if t == 1:
            m.add_constraint(f"EnforceScaledNominalRampDownLimits[{g},{t}]",
                             (q["pg0"] - q["pmin"]) * q["u0"] - PG[g, t] <= q["ramp_dn"])
        else:
            m.add_constraint(f"EnforceScaledNominalRampDownLimits[{g},{t}]", PG[g, t - 1] - PG[g, t] <= q["ramp_dn"])
    for g, t in gt:   # piecewise_production_sum_rule (:1443-1445)
        npc = len(g_[g]["points"]) - 1
        m.add_constraint(f"PiecewiseProductionSum[{g},{t}]", total(PP[g, t, i] for i in range(npc)) == PG[g, t])
    for (g, t, i) in pw:   # piecewise_production_limits_rule (:1447-1449)
        pts = g_[g]["points"]
        m.add_constraint(f"PiecewiseProductionLimits[{g},{t},{i}]", PP[g, t, i] <= (pts[i + 1] - pts[i]) * ON[g, t])
    for g, t in gt:   # piecewise_production_costs_rule (:1452-1458), one row per (g, t)
        pts = g_[g]["points"]
        if len(pts) < 2:
            continue
        m.add_constraint(f"PiecewiseProductionCostsConstr[{g},{t}]",
                         PC[g, t] == total((P.production_cost(g, t, pts[i + 1]) - P.production_cost(g, t, pts[i]))
                                           / (pts[i + 1] - pts[i]) * PP[g, t, i] for i in range(len(pts) - 1)))
    for t in TP:
        m.add_constraint(f"ComputeTotalProductionCost[{t}]", m.TotalProductionCost[t] == total(PC[g, t] for g in G))
    for t in TP:
        m.add_constraint(f"ComputeTotalNoLoadCost[{t}]",
                         m.TotalNoLoadCost[t] == total(g_[g]["minprod"] * ON[g, t] for g in G))
    for g, t in gt:   # startup_match_rule (:1496-1498)
        m.add_constraint(f"StartupMatch[{g},{t}]",
                         total(SI[g, tp, s] for (tp, s) in g_[g]["pairs"] if s == t) <= ST[g, t])
    for g in G:       # shutdown_match_rule (:1503-1513)
        q = g_[g]
        for tp in q["vstp"]:
            begin = [(tp, s) for (a, s) in q["pairs"] if a == tp]
            if tp < 1:
                if begin:
                    m.add_constraint(f"ShutdownMatch[{g},{tp}]", total(SI[g, a, s] for (a, s) in begin) <= 1.0)
            else:
                m.add_constraint(f"ShutdownMatch[{g},{tp}]", total(SI[g, a, s] for (a, s) in begin) <= SP[g, tp])
    for g, t in gt:   # ComputeStartupCost2_rule (:1516-1522)
        q = g_[g]
        lags, sc = q["lags"], q["scosts"]
        e = sc[-1] * ST[g, t]
        for s in range(1, len(lags)):
            e = e + (sc[s - 1] - sc[-1]) * total(SI[g, tp, t] for tp in q["vstp"] if lags[s - 1] <= t - tp < lags[s])
        m.add_constraint(f"ComputeStartupCost2[{g},{t}]", SUC[g, t] == e)
    for g, t in gt:   # compute_shutdown_costs_rule (:1530-1532), ShutdownFixedCost = 0
        m.add_constraint(f"ComputeShutdownCosts[{g},{t}]", SDC[g, t] == 0.0)
    for g in G:       # enforce_up_time_constraints_initial (:1561-1564)
        q = g_[g]
        if q["on_init"] == 0:
            continue
        m.add_constraint(f"EnforceUpTimeConstraintsInitial[{g}]",
                         total(1.0 - ON[g, t] for t in TP if t <= q["on_init"]) == 0.0)
    for g, t in gt:   # unit_start_rule (:1568-1572)
        q = g_[g]
        if t < q["smin_up"]:
            continue
        m.add_constraint(f"unit_start[{g},{t}]",
                         total(ST[g, i] for i in TP if t - q["smin_up"] + 1 <= i <= t) <= ON[g, t])
    for g in G:       # enforce_down_time_constraints_initial (:1582-1585)
        q = g_[g]
        if q["off_init"] == 0:
            continue
        m.add_constraint(f"EnforceDownTimeConstraintsInitial[{g}]",
                         total(ON[g, t] for t in TP if t <= q["off_init"]) == 0.0)
    for g, t in gt:   # unit_stop_rule (:1589-1593)
        q = g_[g]
        if t < q["smin_dn"]:
            continue
        m.add_constraint(f"unit_stop[{g},{t}]",
                         total(SP[g, i] for i in TP if t - q["smin_dn"] + 1 <= i <= t) <= 1.0 - ON[g, t])
    for g, t in gt:   # start_stop_rule (:1603-1606)
        prev = g_[g]["u0"] if t == 1 else ON[g, t - 1]
        m.add_constraint(f"start_stop[{g},{t}]", ON[g, t] - prev == ST[g, t] - SP[g, t])
    # -- objective (:1758-1799): StageCost[FirstStage] + StageCost[SecondStage]
    first = m.add_expression("CommitmentStageCost", total(SUC[g, t] + SDC[g, t] for g, t in gt)
                             + total(g_[g]["minprod"] * P.TPL * ON[g, t] for g, t in gt))
    second = m.add_expression("GenerationStageCost", total(PC[g, t] for g, t in gt)
                              + P.penalty * total(POS["SingleBus", t] + NEG["SingleBus", t] for t in TP)
                              + P.reserve_penalty * total(RS[t] for t in TP))
    m.set_objective(first + second, "min")
    m._mpisppy_node_list = [
        scenario_tree.ScenarioNode(name="ROOT", cond_prob=1.0, stage=1, cost_expression=first,
                                   scen_name_list=None, nonant_list=[m.UnitOn], scen_model=m)]
    if scenario_count is not None:
        m._mpisppy_probability = 1.0 / int(scenario_count)
    return m


def batch_creator(scenario_names, path=None, scenario_count=None):
    """Every scenario at once: the LP of the first one (one model build,
    scenario_creator) with each scenario's wind bounds -- the only data the
    scenarios differ in (NodeN.dat holds Min/MaxNondispatchablePower)."""
    d = _data()
    sset = _scenario_set(path, scenario_count)
    base = scenario_creator(scenario_names[0], path=path, scenario_count=scenario_count)
    one = from_models([scenario_names[0]], [base])
    S = len(scenario_names)
    cols = np.array([base.NondispatchablePowerUsed["WIND", t].col for t in range(1, params().T + 1)])
    l = np.repeat(one.l, S, axis=1)
    u = np.repeat(one.u, S, axis=1)
    for s, nm in enumerate(scenario_names):
        k = sputils.extract_num(nm) - 1
        l[cols, s] = d["scenario_sets"][sset]["wind_min"][k]
        u[cols, s] = d["scenario_sets"][sset]["wind_max"][k]
    prob = None if scenario_count is None else np.full(S, 1.0 / int(scenario_count))
    return BatchData(scenario_names, one.row_ptr, one.col_idx, np.repeat(one.vals, S, axis=1),
                     np.repeat(one.c, S, axis=1), np.repeat(one.const, S), l, u,
                     np.repeat(one.rl, S, axis=1), np.repeat(one.ru, S, axis=1), one.nonant_cols,
                     [one.node_infos[0]] * S, one.sense, prob=prob, var_names=one.var_names)


scenario_creator.batch_creator = batch_creator


def scenario_rhos(scenario, rho_scale_factor=0.1):
    """uc_funcs.py:94-112: rho of UnitOn[g,t] = rho_scale_factor x (the
    production cost at the average power + the minimum production cost).
    Returns [(variable name, rho)] (the nonants named as variables)."""
    P = params()
    out = []
    for t in range(1, P.T + 1):
        for g in P.G:
            q = P.g[g]
            avg = q["pmin"] + (q["pmax"] - q["pmin"]) / 2.0
            cost = P.compute_production_costs(g, t, avg) + q["minprod"]
            out.append((f"UnitOn[{(g, t)}]", rho_scale_factor * cost))
    return out


def scenario_denouement(rank, scenario_name, scenario):
    pass


def all_scenario_names(num_scens):
    """uc_cylinders.py:68: Scenario1 .. ScenarioN."""
    return [f"Scenario{i + 1}" for i in range(num_scens)]
