"""CPU-baseline rank sweep on the GPU box's host (SURVEY 8(d) asks for N =
all physical cores): the oracle PH (oracle/ph_dist.py) on N gloo ranks,
farmer c=1, 200 scenarios, Iter0 + LIMIT PH iterations, N in the argument
list.  The job's cgroup quota (cpu.max) caps the CPUs it may use, so ranks
beyond the quota only time-slice the same CPUs; the solve rate per N shows
where the baseline saturates.  Writes JSON to stdout.

    python tools/cpu_ranks_sweep.py LIMIT N1 N2 ...
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from oracle import ph_dist  # noqa: E402


def main():
    limit = int(sys.argv[1])
    out = {"host": bench.host_cpu_info(), "job_cpus": bench.job_cpus(), "limit": limit, "scenarios": 200, "runs": []}
    for n in map(int, sys.argv[2:]):
        t0 = time.perf_counter()
        r = ph_dist.run(n, 200, crops=1, rho=1.0, convthresh=1e-4, limit=limit)
        wall = time.perf_counter() - t0
        out["runs"].append({"ranks": n, "solves": r["subproblem_solves"],
                            "seconds": round(r["seconds_to_tol"], 3),
                            "solves_per_s": round(r["subproblem_solves"] / r["seconds_to_tol"], 1),
                            "iterations": r["iterations"], "wall_with_startup": round(wall, 1)})
        print(json.dumps(out["runs"][-1]), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":  # (spawned ranks re-import this module)
    main()
