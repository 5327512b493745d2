"""Scenario tree nodes (mirrors ``mpisppy/scenario_tree.py``).

``ScenarioNode`` keeps the reference constructor signature
(``scenario_tree.py:41-95``); ``build_vardatalist`` expands indexed
variables in ``sorted(keys)`` order (``scenario_tree.py:10-38``), which fixes
the nonant order -- and therefore the order of W, xbar and every flat list.
"""
import logging

logger = logging.getLogger("mpisppy_amd.scenario_tree")


def build_vardatalist(self, model, varlist=None):
    """Expand a list of (indexed) variables into scalar VarData objects."""
    if varlist is None:
        raise RuntimeError("varlist is None in scenario_tree.build_vardatalist")
    if not isinstance(varlist, (list, tuple)):
        varlist = [varlist]
    out = []
    for v in varlist:
        if v.is_indexed():
            out.extend(v[i] for i in sorted(v.keys()))
        else:
            out.append(v._scalar() if hasattr(v, "_scalar") else v)
    return out


class ScenarioNode:
    """A non-leaf tree node of one scenario (``scenario_tree.py:41-95``)."""

    def __init__(self, name, cond_prob, stage, cost_expression, scen_name_list,
                 nonant_list, scen_model, nonant_ef_suppl_list=None,
                 parent_name=None):
        self.name = name
        self.cond_prob = cond_prob
        self.stage = stage
        self.cost_expression = cost_expression
        self.nonant_list = nonant_list
        self.nonant_ef_suppl_list = nonant_ef_suppl_list
        self.parent_name = parent_name
        if self.nonant_list is not None:
            self.nonant_vardata_list = build_vardatalist(self, scen_model, self.nonant_list)
        else:
            logger.warning("nonant_list is empty for node %s, No nonanticipativity "
                           "will be enforced at this node by default", name)
            self.nonant_vardata_list = []
        if self.nonant_ef_suppl_list is not None:
            self.nonant_ef_suppl_vardata_list = build_vardatalist(
                self, scen_model, self.nonant_ef_suppl_list)
        else:
            self.nonant_ef_suppl_vardata_list = []

    @property
    def scen_name_list(self):
        raise RuntimeError("The scen name list for a node is not maintained.")
