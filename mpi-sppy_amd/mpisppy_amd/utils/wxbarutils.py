"""W and xbar to / from csv files (``mpisppy/utils/wxbarutils.py``).

Same file formats and checks as the reference:

* one master W file, rows ``scenario_name,variable_name,weight`` (written by
  rank 0 after a gather, appended; ``wxbarutils.py:40-79``), or one file per
  scenario ``<scenario_name>_weights.csv`` with rows ``variable_name,weight``;
* the xbar file, rows ``variable_name,value`` (``wxbarutils.py:264-284``);
* lines starting with ``#`` are comments; variable names may contain commas;
* reading checks for missing / extra variables and the dual feasibility of
  the weights, sum_s p_s W_s = 0 within 1e-7 (``wxbarutils.py:212-261``).

Here W and xbar live on the device as [K][S] tensors (scenario-fastest);
these helpers move them through host numpy arrays.
"""
import os

import numpy as np
import torch


def _local_W(PHB):
    return PHB.W.view(PHB.K, PHB.S_loc).cpu().numpy()       # [K][S]


def write_W_to_file(PHB, fname, sep_files=False):
    """wxbarutils.py:40-79."""
    names = PHB.nonant_names()
    W = _local_W(PHB)
    if sep_files:
        os.makedirs(fname, exist_ok=True)
        for s, sname in enumerate(PHB.local_scenario_names):
            with open(os.path.join(fname, sname + "_weights.csv"), "w") as f:
                for k, vname in enumerate(names):
                    f.write(",".join([vname, str(float(W[k, s]))]) + "\n")
        return
    local = [(sname, names[k], float(W[k, s]))
             for s, sname in enumerate(PHB.local_scenario_names) for k in range(PHB.K)]
    allw = PHB.comm.gather_object(local)
    if PHB.cylinder_rank == 0:
        with open(fname, "a") as f:
            for part in allw:
                for sname, vname, val in part:
                    f.write(",".join([sname, vname, str(val)]) + "\n")


def _parse_W_csv_single(fname):
    """wxbarutils.py:123-143."""
    if not os.path.exists(fname):
        raise RuntimeError("Could not find file {fn}".format(fn=fname))
    results = {}
    with open(fname, "r") as f:
        for line in f:
            if line.startswith("#"):
                continue
            parts = line.split(",")
            results[",".join(parts[:-1])] = float(parts[-1])
    return results


def _parse_W_csv(fname, scenario_names_local, scenario_names_global, rank):
    """wxbarutils.py:145-210."""
    results = {}
    seen = {name: False for name in scenario_names_local}
    glob = set(scenario_names_global)
    loc = set(scenario_names_local)
    with open(fname, "r") as f:
        for line in f:
            if line.startswith("#"):
                continue
            parts = line.split(",")
            sname = parts[0]
            vname = ",".join(parts[1:-1])
            wval = float(parts[-1])
            if sname not in glob:
                if rank == 0:
                    print("WARNING: Ignoring unknown scenario name", sname)
                continue
            if sname not in loc:
                continue
            results.setdefault(sname, {})[vname] = wval
            seen[sname] = True
    missing = [name for name, ok in seen.items() if not ok]
    if missing:
        raise RuntimeError("rank " + str(rank) + " could not find the following "
                           "scenarios in the provided weight file: " + ", ".join(missing))
    return results


def _check_W(w_val_dict, PHB, rank):
    """wxbarutils.py:212-261: missing variables raise, extra ones are dropped
    with a message, and sum_s p_s W_s must vanish (1e-7)."""
    vn_model = set(PHB.nonant_names())
    for sname in PHB.local_scenario_names:
        provided = set(w_val_dict[sname].keys())
        diff = vn_model.difference(provided)
        if diff:
            raise RuntimeError(sname + " is missing the following variables: " + ", ".join(sorted(diff)))
        diff = provided.difference(vn_model)
        if diff:
            print("Removing unknown variables:", ", ".join(sorted(diff)))
            for vname in diff:
                w_val_dict[sname].pop(vname, None)
    names = PHB.nonant_names()
    local = np.zeros(len(names))
    for s, sname in enumerate(PHB.local_scenario_names):
        local += PHB.local_prob[s] * np.array([w_val_dict[sname][v] for v in names])
    tot = PHB.comm.allreduce_host(list(local))
    for k, vname in enumerate(names):
        if abs(tot[k]) > 1e-7:
            raise RuntimeError("Provided weights do not satisfy dual feasibility: "
                               "\\sum_{scenarios} prob(s) * w(s) != 0. Error on variable " + vname)


def set_W_from_file(fname, PHB, rank, sep_files=False):
    """wxbarutils.py:81-121."""
    if sep_files:
        w_val_dict = {sname: _parse_W_csv_single(os.path.join(fname, sname + "_weights.csv"))
                      for sname in PHB.local_scenario_names}
    else:
        w_val_dict = _parse_W_csv(fname, PHB.local_scenario_names, PHB.all_scenario_names, rank)
    _check_W(w_val_dict, PHB, rank)
    names = PHB.nonant_names()
    W = np.array([[w_val_dict[sname][v] for sname in PHB.local_scenario_names] for v in names])
    PHB.W.copy_(torch.as_tensor(W.reshape(-1), dtype=torch.float64, device=PHB.W.device))


def write_xbar_to_file(PHB, fname):
    """wxbarutils.py:264-284: rank 0 writes its first scenario's xbars."""
    if PHB.cylinder_rank != 0:
        return
    xb = PHB.xbar.view(PHB.K, PHB.S_loc)[:, 0].cpu().numpy()
    with open(fname, "a") as f:
        for vname, val in zip(PHB.nonant_names(), xb):
            f.write(",".join([vname, str(float(val))]) + "\n")


def _parse_xbar_csv(fname):
    """wxbarutils.py:310-344."""
    results = {}
    with open(fname, "r") as f:
        for line in f:
            if line.startswith("#"):
                continue
            parts = line.split(",")
            results[",".join(parts[:-1])] = float(parts[-1])
    return results


def _check_xbar(xbar_val_dict, PHB):
    """wxbarutils.py:346-366."""
    var_names = set(PHB.nonant_names())
    provided = set(xbar_val_dict.keys())
    missing = var_names.difference(provided)
    if missing:
        raise RuntimeError("Could not find the following required variable values in the "
                           "provided input file: " + ", ".join(sorted(missing)))
    extra = provided.difference(var_names)
    if extra:
        print("Ignoring the following variables values provided in the input file: "
              + ", ".join(sorted(extra)))


def set_xbar_from_file(fname, PHB):
    """wxbarutils.py:286-308: xbar from the file, xsqbar = xbar^2, for every
    local scenario (the file holds one value per nonant variable name)."""
    xbar_val_dict = _parse_xbar_csv(fname)
    if PHB.cylinder_rank == 0:
        _check_xbar(xbar_val_dict, PHB)
    vals = np.array([xbar_val_dict[v] for v in PHB.nonant_names()])
    xb = np.repeat(vals[:, None], PHB.S_loc, axis=1).reshape(-1)
    t = torch.as_tensor(xb, dtype=torch.float64, device=PHB.xbar.device)
    PHB.xbar.copy_(t)
    PHB.xsqbar.copy_(t * t)
