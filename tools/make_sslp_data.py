"""Convert the reference's sslp .dat files (examples/sslp/data/<inst>/
scenariodata/Scenario*.dat, AMPL/Pyomo data format) into the compact JSON
the sslp example reads (mpisppy_amd/examples/data/sslp.json).

    python tools/make_sslp_data.py /root/reference/examples/sslp/data

The instances share NumServers, NumClients, Capacity, FixedCost, Revenue and
Demand per (servers, clients) size; scenarios differ only in ClientPresent.
This script checks that and stores the shared data once per size plus the
ClientPresent rows of every scenario of every instance.
"""
import glob
import json
import os
import re
import sys


def parse_dat(path):
    txt = open(path).read()
    out = {}
    for stmt in txt.split(";"):
        stmt = stmt.strip()
        if not stmt.startswith("param"):
            continue
        head, _, body = stmt.partition(":=") if ":=" in stmt.split("\n")[0] else (None, None, None)
        if head is not None:  # scalar or 1-d: "param X := v" or "param X:= k v k v"
            name = head.split()[1].strip()
            toks = body.split()
            if len(toks) == 1:
                out[name] = float(toks[0])
            else:
                out[name] = {int(toks[i]): float(toks[i + 1]) for i in range(0, len(toks), 2)}
            continue
        # 2-d table: "param X:\n c1 c2 ... :=\n r v v v ..."
        lines = stmt.split("\n")
        name = lines[0].split()[1].rstrip(":")
        hdr, _, rest = stmt.partition(":=")
        cols = [int(t) for t in hdr.split("\n", 1)[1].split()]
        tab = {}
        for line in rest.strip().split("\n"):
            toks = line.split()
            if not toks:
                continue
            r = int(toks[0])
            for c, v in zip(cols, toks[1:]):
                tab[(r, c)] = float(v)
        out[name] = tab
    return out


def main():
    root = sys.argv[1]
    shared = {}
    instances = {}
    for inst in sorted(os.listdir(root)):
        d = os.path.join(root, inst, "scenariodata")
        files = [p for p in glob.glob(os.path.join(d, "Scenario*.dat"))
                 if re.search(r"Scenario\d+\.dat$", p)]
        files.sort(key=lambda p: int(re.findall(r"(\d+)\.dat$", p)[0]))
        present = []
        for f in files:
            p = parse_dat(f)
            ns, nc = int(p["NumServers"]), int(p["NumClients"])
            key = f"{ns}_{nc}"
            base = {"NumServers": ns, "NumClients": nc, "Capacity": p["Capacity"],
                    "FixedCost": [p["FixedCost"].get(j, 0.0) for j in range(1, ns + 1)],
                    "Revenue": [[p["Revenue"].get((i, j), 0.0) for j in range(1, ns + 1)]
                                for i in range(1, nc + 1)],
                    "Demand": [[p["Demand"].get((i, j), 0.0) for j in range(1, ns + 1)]
                               for i in range(1, nc + 1)]}
            if key in shared:
                if shared[key] != base:
                    raise SystemExit(f"{f}: shared data differ from the other scenarios")
            else:
                shared[key] = base
            cp = p.get("ClientPresent", {})
            present.append([int(cp.get(i, 1.0)) for i in range(1, nc + 1)])
        instances[inst] = {"size": key, "ClientPresent": present}
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "mpi-sppy_amd", "mpisppy_amd", "examples", "data", "sslp.json")
    with open(out, "w") as f:
        json.dump({"source": "mpi-sppy examples/sslp/data/*/scenariodata/Scenario*.dat "
                             "(converted by tools/make_sslp_data.py)",
                   "sizes": shared, "instances": instances}, f, separators=(",", ":"))
    print(out, {k: len(v["ClientPresent"]) for k, v in instances.items()})


if __name__ == "__main__":
    main()
