"""Convert the reference's UC data (paperruns/larger_uc: the WECC-240
RootNode.dat and the NodeN.dat wind scenarios) into the compact JSON the UC
example reads (data only: every number as the .dat files hold it).

    python tools/make_uc_data.py /root/reference/paperruns/larger_uc \\
        mpi-sppy_amd/mpisppy_amd/examples/data/uc_wecc240.json

Root: the generators' parameter table, piecewise cost points / values,
startup lags / costs, demand, reserve requirement, penalties, horizon.
Scenarios: per NodeN.dat of 1000scenarios_wind the 48 (min, max)
nondispatchable (wind) power bounds; 3scenarios_wind's files (50 nodes)
are kept as a second set.
"""
import json
import os
import re
import sys


def _blocks(text):
    """Statements of a .dat file (comments dropped), split at ';'."""
    text = "\n".join(ln.split("#", 1)[0] for ln in text.splitlines())
    return [b.strip() for b in text.split(";") if b.strip()]


def parse_root(path):
    out = {"gen_table": {}, "piecewise_points": {}, "piecewise_values": {}, "startup_lags": {},
           "startup_costs": {}, "demand": {}, "reserve": {}}
    for b in _blocks(open(path).read()):
        toks = b.split()
        if b.startswith("param LoadMismatchPenalty"):
            out["LoadMismatchPenalty"] = float(toks[-1])
        elif b.startswith("param NumTimePeriods"):
            out["NumTimePeriods"] = int(toks[-1])
        elif b.startswith("param TimePeriodLength"):
            out["TimePeriodLength"] = float(toks[-1])
        elif b.startswith("set ThermalGenerators ") or b.startswith("set ThermalGenerators:"):
            out["ThermalGenerators"] = b.split(":=", 1)[1].split()
        elif b.startswith("set QuickStartGenerators"):
            out["QuickStartGenerators"] = b.split(":=", 1)[1].split()
        elif b.startswith("set Buses"):
            out["Buses"] = b.split(":=", 1)[1].split()
        elif b.startswith("set NondispatchableGeneratorsAtBus"):
            out["Nondispatchable"] = b.split(":=", 1)[1].split()
        elif b.startswith("param: PowerGeneratedT0"):
            head, body = b.split(":=", 1)
            cols = head.split()[1:]
            vals = body.split()
            w = len(cols) + 1
            for i in range(0, len(vals), w):
                out["gen_table"][vals[i]] = dict(zip(cols, map(float, vals[i + 1:i + w])))
        elif b.startswith("param: ReserveRequirement"):
            vals = b.split(":=", 1)[1].split()
            for i in range(0, len(vals), 2):
                out["reserve"][int(vals[i])] = float(vals[i + 1])
        elif b.startswith("param: Demand"):
            vals = b.split(":=", 1)[1].split()
            for i in range(0, len(vals), 3):
                out["demand"][int(vals[i + 1])] = float(vals[i + 2])
        else:
            m = re.match(r"set (CostPiecewisePoints|CostPiecewiseValues|StartupLags|StartupCosts)\[(.+?)\]", b)
            if m:
                key = {"CostPiecewisePoints": "piecewise_points", "CostPiecewiseValues": "piecewise_values",
                       "StartupLags": "startup_lags", "StartupCosts": "startup_costs"}[m.group(1)]
                vals = b.split(":=", 1)[1].split()
                conv = int if key == "startup_lags" else float
                out[key][m.group(2)] = [conv(v) for v in vals]
    T = out["NumTimePeriods"]
    out["demand"] = [out["demand"][t] for t in range(1, T + 1)]
    out["reserve"] = [out["reserve"].get(t, 0.0) for t in range(1, T + 1)]
    return out


def parse_node(path, T):
    lo, hi = [0.0] * T, [0.0] * T
    for b in _blocks(open(path).read()):
        which = lo if b.startswith("param MinNondispatchablePower") else \
            hi if b.startswith("param MaxNondispatchablePower") else None
        if which is None:
            continue
        vals = b.split(":=", 1)[1].split()
        for i in range(0, len(vals), 3):
            which[int(vals[i + 1]) - 1] = float(vals[i + 2])
    return lo, hi


def main():
    src, dst = sys.argv[1], sys.argv[2]
    root = parse_root(os.path.join(src, "1000scenarios_wind", "RootNode.dat"))
    T = root["NumTimePeriods"]
    sets = {}
    for d, n in (("1000scenarios_wind", 1000), ("3scenarios_wind", 50)):
        lo, hi = [], []
        for k in range(1, n + 1):
            a, b = parse_node(os.path.join(src, d, f"Node{k}.dat"), T)
            lo.append(a)
            hi.append(b)
        sets[d] = {"wind_min": lo, "wind_max": hi}
    root["scenario_sets"] = sets
    root["source"] = ("/root/reference/paperruns/larger_uc/{1000,3}scenarios_wind/RootNode.dat + NodeN.dat "
                      "(data of the reference, converted by tools/make_uc_data.py)")
    with open(dst, "w") as f:
        json.dump(root, f, separators=(",", ":"))
    print(dst, os.path.getsize(dst), "bytes;", len(root["ThermalGenerators"]), "generators,", T, "periods")


if __name__ == "__main__":
    main()
