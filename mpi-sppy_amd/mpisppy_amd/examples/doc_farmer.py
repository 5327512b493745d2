"""The textbook farmer of the reference docs (``doc/src/examples.rst:50-175``)."""
from ..model import LinearModel
from ..utils import sputils

YIELDS = {"good": [3, 3.6, 24], "average": [2.5, 3, 20], "bad": [2, 2.4, 16]}


def build_model(yields):
    m = LinearModel("farmer")
    m.add_var("X", ["WHEAT", "CORN", "BEETS"], lb=0.0)
    m.add_var("Y", ["WHEAT", "CORN"], lb=0.0)
    m.add_var("W", ["WHEAT", "CORN", "BEETS_FAVORABLE", "BEETS_UNFAVORABLE"], lb=0.0,
              ub=lambda k: 6000.0 if k == "BEETS_FAVORABLE" else None)
    X, Y, W = m.X, m.Y, m.W
    m.add_expression("PLANTING_COST", 150 * X["WHEAT"] + 230 * X["CORN"] + 260 * X["BEETS"])
    m.add_expression("PURCHASE_COST", 238 * Y["WHEAT"] + 210 * Y["CORN"])
    m.add_expression("SALES_REVENUE", 170 * W["WHEAT"] + 150 * W["CORN"]
                     + 36 * W["BEETS_FAVORABLE"] + 10 * W["BEETS_UNFAVORABLE"])
    m.set_objective(m.PLANTING_COST + m.PURCHASE_COST - m.SALES_REVENUE, "min")
    m.add_constraint("CONSTR[1]", X["WHEAT"] + X["CORN"] + X["BEETS"] <= 500)
    m.add_constraint("CONSTR[2]", yields[0] * X["WHEAT"] + Y["WHEAT"] - W["WHEAT"] >= 200)
    m.add_constraint("CONSTR[3]", yields[1] * X["CORN"] + Y["CORN"] - W["CORN"] >= 240)
    m.add_constraint("CONSTR[4]", yields[2] * X["BEETS"] - W["BEETS_FAVORABLE"]
                     - W["BEETS_UNFAVORABLE"] >= 0)
    return m


def scenario_creator(scenario_name):
    if scenario_name not in YIELDS:
        raise ValueError("Unrecognized scenario name")
    model = build_model(YIELDS[scenario_name])
    sputils.attach_root_node(model, model.PLANTING_COST, [model.X])
    model._mpisppy_probability = 1.0 / 3
    return model
