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


def spin_the_wheel(hub_dict, list_of_spoke_dict, comm_world=None):
    """sputils.py:24-131, in process: every rank builds the hub's opt object
    and every spoke's (each over the rank's own scenarios, each with its own
    device batch), the spokes are attached to the hub, and the hub runs PH,
    syncing the spokes every ``hub_kwargs["sync_every"]`` iterations.
    Returns (hub, hub_dict) like the reference's (spcomm, opt_dict)."""
    if "hub_class" not in hub_dict:
        raise RuntimeError("The hub_dict must contain a 'hub_class' key specifying the hub class to use")
    if "opt_class" not in hub_dict:
        raise RuntimeError("The hub_dict must contain an 'opt_class' key specifying the SPBase "
                           "class to use (e.g. PHBase, etc.)")
    hub_dict.setdefault("hub_kwargs", {})
    hub_dict.setdefault("opt_kwargs", {})
    for sd in list_of_spoke_dict:
        if "spoke_class" not in sd:
            raise RuntimeError("Each spoke_dict must contain a 'spoke_class' key specifying the "
                               "spoke class to use")
        if "opt_class" not in sd:
            raise RuntimeError("Each spoke_dict must contain an 'opt_class' key specifying the "
                               "SPBase class to use (e.g. PHBase, etc.)")
        sd.setdefault("spoke_kwargs", {})
        sd.setdefault("opt_kwargs", {})
    kw = dict(hub_dict["opt_kwargs"])
    if comm_world is not None:
        kw["mpicomm"] = comm_world
    opt = hub_dict["opt_class"](**kw)
    spokes = []
    for sd in list_of_spoke_dict:
        skw = dict(sd["opt_kwargs"])
        if comm_world is not None:
            skw["mpicomm"] = comm_world
        spokes.append(sd["spoke_class"](sd["opt_class"](**skw), **sd["spoke_kwargs"]))
    hub = hub_dict["hub_class"](opt, spokes, **hub_dict["hub_kwargs"])
    hub.main()
    hub.hub_finalize()
    return hub, hub_dict
