"""The scalable farmer (``examples/farmer/farmer.py`` of the reference).

``scenario_creator`` builds one scenario as a LinearModel with the reference's
variables, constraints, nonant node and RNG stream; ``batch_creator`` builds
the scenario-batched arrays for many scenarios at once with numpy (same
numbers, no per-scenario model objects) -- the path used at 10k scenarios.
"""
import numpy as np

from ..model import LinearModel
from .. import scenario_tree
from ..utils import sputils
from ..batch import BatchData, NodeInfo

CROP_BASES = ["WHEAT", "CORN", "SUGAR_BEETS"]
PRICE_QUOTA = {"WHEAT": 100000.0, "CORN": 100000.0, "SUGAR_BEETS": 6000.0}
SUB_QUOTA_PRICE = {"WHEAT": 170.0, "CORN": 150.0, "SUGAR_BEETS": 36.0}
SUPER_QUOTA_PRICE = {"WHEAT": 0.0, "CORN": 0.0, "SUGAR_BEETS": 10.0}
CATTLE_FEED = {"WHEAT": 200.0, "CORN": 240.0, "SUGAR_BEETS": 0.0}
PURCHASE_PRICE = {"WHEAT": 238.0, "CORN": 210.0, "SUGAR_BEETS": 100000.0}
PLANTING_COST = {"WHEAT": 150.0, "CORN": 230.0, "SUGAR_BEETS": 260.0}
YIELD = {  # farmer.py:142-148
    "BelowAverageScenario": {"WHEAT": 2.0, "CORN": 2.4, "SUGAR_BEETS": 16.0},
    "AverageScenario": {"WHEAT": 2.5, "CORN": 3.0, "SUGAR_BEETS": 20.0},
    "AboveAverageScenario": {"WHEAT": 3.0, "CORN": 3.6, "SUGAR_BEETS": 24.0},
}
BASENAMES = ["BelowAverageScenario", "AverageScenario", "AboveAverageScenario"]


def crops(crops_multiplier):
    """CROPS in set order: WHEAT0, CORN0, SUGAR_BEETS0, WHEAT1, ... (farmer.py:98-104)."""
    return [b + str(i) for i in range(crops_multiplier) for b in CROP_BASES]


def yields(scennum, crops_multiplier=1):
    """Per-crop yields of scenario ``scennum`` (farmer.py:44-54,150-156): the
    stream is seeded with the scenario number and, for groupnum > 0, one
    uniform draw per crop in CROPS order is added to the base yield."""
    base = BASENAMES[scennum % 3]
    groupnum = scennum // 3
    stream = np.random.RandomState(scennum)
    out = np.empty(3 * crops_multiplier)
    for k, crop in enumerate(crops(crops_multiplier)):
        y = YIELD[base][crop.rstrip("0123456789")]
        out[k] = y + stream.rand() if groupnum != 0 else y
    return out


def scenario_creator(scenario_name, use_integer=False, sense="min", crops_multiplier=1,
                     num_scens=None):
    """One farmer scenario (farmer.py:24-82; model farmer.py:84-223)."""
    if use_integer:
        raise NotImplementedError("integer farmer is a MIP; the PDHG hot path solves LP/QP")
    if sense not in ("min", "max"):
        raise ValueError("Model sense Not recognized")
    scennum = sputils.extract_num(scenario_name)
    cm = crops_multiplier
    CROPS = crops(cm)
    Y = dict(zip(CROPS, yields(scennum, cm)))
    base = lambda c: c.rstrip("0123456789")
    m = LinearModel(scenario_name)
    total = 500.0 * cm
    m.add_var("DevotedAcreage", CROPS, lb=0.0, ub=total)
    m.add_var("QuantitySubQuotaSold", CROPS, lb=0.0)
    m.add_var("QuantitySuperQuotaSold", CROPS, lb=0.0)
    m.add_var("QuantityPurchased", CROPS, lb=0.0)
    DA, QSUB, QSUP, QP = (m.DevotedAcreage, m.QuantitySubQuotaSold,
                          m.QuantitySuperQuotaSold, m.QuantityPurchased)
    m.add_constraint("ConstrainTotalAcreage", sum(DA[c] for c in CROPS) <= total)
    for c in CROPS:
        m.add_constraint(f"EnforceCattleFeedRequirement[{c}]",
                         Y[c] * DA[c] + QP[c] - QSUB[c] - QSUP[c] >= CATTLE_FEED[base(c)])
    for c in CROPS:
        m.add_constraint(f"LimitAmountSold[{c}]", QSUB[c] + QSUP[c] - Y[c] * DA[c] <= 0.0)
    for c in CROPS:
        m.add_constraint(f"EnforceQuotas[{c}]", 1.0 * QSUB[c], lo=0.0, hi=PRICE_QUOTA[base(c)])
    first = m.add_expression("FirstStageCost", sum(PLANTING_COST[base(c)] * DA[c] for c in CROPS))
    second = m.add_expression(
        "SecondStageCost",
        sum(PURCHASE_PRICE[base(c)] * QP[c] for c in CROPS)
        - sum(SUB_QUOTA_PRICE[base(c)] * QSUB[c] for c in CROPS)
        - sum(SUPER_QUOTA_PRICE[base(c)] * QSUP[c] for c in CROPS))
    if sense == "min":
        m.set_objective(first + second, "min")
    else:
        m.set_objective(-first - second, "max")
    m._mpisppy_node_list = [
        scenario_tree.ScenarioNode(name="ROOT", cond_prob=1.0, stage=1,
                                   cost_expression=m.FirstStageCost, scen_name_list=None,
                                   nonant_list=[m.DevotedAcreage], scen_model=m)
    ]
    if num_scens is not None:
        m._mpisppy_probability = 1.0 / num_scens
    return m


def batch_creator(scenario_names, sense="min", crops_multiplier=1, num_scens=None,
                  use_integer=False):
    """All ``scenario_names`` at once as a :class:`BatchData` (same numbers
    as ``scenario_creator``; column order DA, QSUB, QSUP, QP by CROPS)."""
    if use_integer:
        raise NotImplementedError("integer farmer is a MIP")
    cm = crops_multiplier
    CROPS = crops(cm)
    nc = len(CROPS)
    S = len(scenario_names)
    n = 4 * nc
    DA = np.arange(nc); QSUB = nc + DA; QSUP = 2 * nc + DA; QP = 3 * nc + DA
    bases = [c.rstrip("0123456789") for c in CROPS]
    Y = np.stack([yields(sputils.extract_num(nm), cm) for nm in scenario_names], axis=1)  # [nc][S]
    # pattern, row by row, columns sorted inside a row (as LinearModel does)
    rows = [[(int(j), None) for j in DA]]                                   # total acreage
    for k in range(nc):
        rows.append(sorted([(int(DA[k]), ("Y", k)), (int(QSUB[k]), -1.0),
                            (int(QSUP[k]), -1.0), (int(QP[k]), 1.0)]))
    for k in range(nc):
        rows.append(sorted([(int(DA[k]), ("-Y", k)), (int(QSUB[k]), 1.0), (int(QSUP[k]), 1.0)]))
    for k in range(nc):
        rows.append([(int(QSUB[k]), 1.0)])
    row_ptr = np.zeros(len(rows) + 1, dtype=np.int32)
    col_idx, vals = [], []
    for i, r in enumerate(rows):
        for j, v in r:
            col_idx.append(j)
            if v is None:
                vals.append(np.ones(S))
            elif isinstance(v, tuple):
                vals.append(Y[v[1]] if v[0] == "Y" else -Y[v[1]])
            else:
                vals.append(np.full(S, v))
        row_ptr[i + 1] = len(col_idx)
    vals = np.stack(vals, axis=0)
    m_ = len(rows)
    cvec = np.zeros(n)
    for k, b in enumerate(bases):
        cvec[DA[k]] = PLANTING_COST[b]
        cvec[QP[k]] = PURCHASE_PRICE[b]
        cvec[QSUB[k]] = -SUB_QUOTA_PRICE[b]
        cvec[QSUP[k]] = -SUPER_QUOTA_PRICE[b]
    # min form: a maximize model's objective is -(first+second); negated -> same c
    c = np.repeat(cvec[:, None], S, axis=1)
    lvec = np.zeros(n)
    uvec = np.full(n, np.inf)
    uvec[DA] = 500.0 * cm
    rl = np.empty(m_); ru = np.empty(m_)
    rl[0], ru[0] = -np.inf, 500.0 * cm
    for k, b in enumerate(bases):
        rl[1 + k], ru[1 + k] = CATTLE_FEED[b], np.inf
        rl[1 + nc + k], ru[1 + nc + k] = -np.inf, 0.0
        rl[1 + 2 * nc + k], ru[1 + 2 * nc + k] = 0.0, PRICE_QUOTA[b]
    order = sorted(range(nc), key=lambda k: CROPS[k])       # sorted nonant keys
    nonant_cols = DA[order]
    names = ([f"DevotedAcreage[{c}]" for c in CROPS] + [f"QuantitySubQuotaSold[{c}]" for c in CROPS]
             + [f"QuantitySuperQuotaSold[{c}]" for c in CROPS] + [f"QuantityPurchased[{c}]" for c in CROPS])
    infos = [NodeInfo([("ROOT", 1.0, nc)])] * S
    prob = None if num_scens is None else np.full(S, 1.0 / num_scens)
    return BatchData(scenario_names, row_ptr, np.asarray(col_idx), vals, c, np.zeros(S),
                     np.repeat(lvec[:, None], S, 1), np.repeat(uvec[:, None], S, 1),
                     np.repeat(rl[:, None], S, 1), np.repeat(ru[:, None], S, 1),
                     nonant_cols, infos, sense, prob=prob, var_names=names)


scenario_creator.batch_creator = batch_creator


def scenario_denouement(rank, scenario_name, scenario):
    pass
