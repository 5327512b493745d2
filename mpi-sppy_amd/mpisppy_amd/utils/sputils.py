"""Utilities kept from ``mpisppy/utils/sputils.py`` that the hot path needs."""
import re

from .. import scenario_tree


def extract_num(string):
    """Trailing integer of a name, e.g. scenario324 -> 324 (``sputils.py:414-423``)."""
    return int(re.compile(r"(\d+)$").search(string).group(1))


def rank_slices(num_scens, n_proc):
    """Contiguous scenario slices per rank (``sputils.py:619-628``):
    ``avg = S/n``; rank i owns ``range(int(i*avg), int((i+1)*avg))``."""
    if n_proc == 1:
        return [list(range(num_scens))]
    avg = num_scens / n_proc
    return [list(range(int(i * avg), int((i + 1) * avg))) for i in range(n_proc)]


def scen_names_to_ranks(all_scenario_names, n_proc):
    """(slices, rank of each scenario index) -- ``_ScenTree.scen_names_to_ranks``."""
    slices = rank_slices(len(all_scenario_names), n_proc)
    ranks = [r for r, sl in enumerate(slices) for _ in sl]
    return slices, ranks


def attach_root_node(model, firstobj, varlist, nonant_ef_suppl_list=None):
    """``sputils.py:665-681``: a two-stage scenario's single ROOT node."""
    model._mpisppy_node_list = [
        scenario_tree.ScenarioNode("ROOT", 1.0, 1, firstobj, None, varlist, model,
                                   nonant_ef_suppl_list=nonant_ef_suppl_list)
    ]


def option_string_to_dict(ostr):
    """``sputils.option_string_to_dict``: "k=v k2=v2" -> dict (values as float if possible)."""
    out = {}
    if ostr is None:
        return out
    for tok in ostr.split():
        if "=" in tok:
            k, v = tok.split("=", 1)
            try:
                v = float(v) if ("." in v or "e" in v.lower()) else int(v)
            except ValueError:
                pass
            out[k] = v
        else:
            out[tok] = None
    return out
