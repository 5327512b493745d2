"""Per-kernel HBM bytes per launch from rocprofv3 PMC passes of bench.py.

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR STATS_DIR OUT.json WORKLOAD [WINDOW]

FETCH_DIR / WRITE_DIR: `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
output directories (separate passes, csv).  FETCH_SIZE and WRITE_SIZE are in
kB per dispatch; per MI355X_MICROARCH.md (HBM section) FETCH_SIZE on gfx950
reports half the bytes of coalesced reads, so it is doubled here.
STATS_DIR: the `--kernel-trace --stats` run (kernel time per launch).

WORKLOAD names the one workload the profiled command ran (each profiled
bench command runs ONE config: `--tol-run 0 --hbm-crops 0 --sslp-scens 0`
for the farmer lines, `--crops 0 --hbm-crops 0 --sslp-scens N` style runs
for sslp); the summary refuses a window whose kernel instances do not belong
to it (a window that caught another config's launches is what mislabelled
the round-2 profiles):

  farmer10k_c1    active_set_kernel exactly once per solve, no mid-size kernel
  farmer10k_c100  mid_kernel<512, 3, 2> / mid_polish_kernel<512, 3, 2> only
                  (n = 1200, m = 901; 512-thread instances since round 3),
                  no active_set_kernel
  farmer1k_c1000  big_kernel / big_polish_kernel (the big path: n = 12,000,
                  m = 9,001), no one-wave or mid-size kernel
  sslp10k         mid_kernel<512, 2, 1> / mid_polish_kernel<512, 2, 1> only
                  (n = 705, m = 60)

Window "first": the launches up to the first `summary_kernel` dispatch (the
Iter0 solve, e.g. F4's streaming PDHG).
Window N: the launches after the (N+1)-th last `summary_kernel` dispatch,
i.e. the last WINDOW solve calls (one summary kernel closes each solve) --
the eagerly launched PH iterations whose HIP-event times give the bench
line's `achieved`, so traffic and algorithmic bytes describe the same
launches.  Kernels are named by their function name (template arguments
dropped, kept under "instances"); `launches_per_solve` = launches in the
window / WINDOW.  VGPR count and scratch (spill) bytes per lane come from
the same records.
"""
import csv
import glob
import json
import os
import re
import sys

_NAME = re.compile(r"::(\w+)\s*[<(]")
_INST = re.compile(r"::(\w+\s*<[^>]*>)")

WORKLOADS = {
    "farmer10k_c1": {"scenarios_per_rank": 10000, "crops_multiplier": 1,
                     "require": {}, "require_any": ["active_set_kernel", "active_set_g_kernel"],
                     "forbid": ["mid_kernel", "mid_polish_kernel"],
                     "once_per_solve": ["active_set_kernel", "active_set_g_kernel"]},
    "farmer10k_c100": {"scenarios_per_rank": 10000, "crops_multiplier": 100,
                       "require": {"mid_kernel": "mid_kernel<512, 3, 2>",
                                   "mid_polish_kernel": "mid_polish_kernel<512, 3, 2>"},
                       "forbid": ["active_set_kernel"], "once_per_solve": []},
    "farmer1k_c1000": {"scenarios_per_rank": 1000, "crops_multiplier": 1000,
                       "require": {"big_kernel": None, "big_polish_kernel": "big_polish_kernel<false>"},
                       "forbid": ["active_set_kernel", "mid_kernel"], "once_per_solve": []},
    "sslp10k": {"scenarios_per_rank": 10000, "crops_multiplier": None,
                "require": {"mid_kernel": "mid_kernel<1024, 1, 1>",
                            "mid_polish_kernel": "mid_polish_kernel<1024, 1, 1>"},
                "forbid": ["active_set_kernel"], "once_per_solve": []},
}


def short(name):
    m = _NAME.search(name)
    if m:
        return m.group(1)
    return name.split("(")[0].strip()


def instance(name):
    m = _INST.search(name)
    return m.group(1) if m else short(name)


def _rows(d, pattern):
    f = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    if not f:
        raise SystemExit(f"pmc_summary: no {pattern} under {d}")
    rows = list(csv.DictReader(open(f[0])))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def _window(rows, window):
    """(first, last] dispatch ids of the window: the last `window` solve
    calls, or with window "first" the process's first solve call (Iter0)."""
    # a solve call ends with summary_kernel, or (the fused single-rank
    # pass, round 5) with finish_kernel
    summ = sorted({int(r["Dispatch_Id"]) for r in rows
                   if short(r["Kernel_Name"]) in ("summary_kernel", "finish_kernel")})
    if window == "first":
        if not summ:
            raise SystemExit("pmc_summary: no solve call recorded")
        return -1, summ[0]
    if len(summ) <= window:
        raise SystemExit(f"pmc_summary: only {len(summ)} solve calls recorded, window {window}")
    return summ[-window - 1], 1 << 62


def per_kernel(d, counter, window):
    rows = [r for r in _rows(d, "*counter_collection.csv") if r["Counter_Name"] == counter]
    w0, w1 = _window(rows, window)
    vals, meta, inst = {}, {}, {}
    for r in rows:
        if not (w0 < int(r["Dispatch_Id"]) <= w1):
            continue
        k = short(r["Kernel_Name"])
        vals.setdefault(k, []).append(float(r["Counter_Value"]))
        inst.setdefault(k, set()).add(instance(r["Kernel_Name"]))
        meta[k] = {"vgpr": int(r["VGPR_Count"]), "accum_vgpr": int(r["Accum_VGPR_Count"]),
                   "scratch_bytes_per_lane": int(r["Scratch_Size"]),
                   "lds_bytes": int(r["LDS_Block_Size"]), "workgroup": int(r["Workgroup_Size"])}
    return {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}, meta, inst


def validate(tag, res, inst):
    """Refuse a window that holds another workload's kernels."""
    w = WORKLOADS[tag]
    ks = res["kernels"]
    for k, want in w["require"].items():
        if k not in ks:
            raise SystemExit(f"pmc_summary: workload {tag} needs {k} in the window; found {sorted(ks)}")
        if want is not None and inst.get(k) != {want}:
            raise SystemExit(f"pmc_summary: workload {tag} needs only {want}; the window holds "
                             f"{sorted(inst.get(k, []))}")
    if w.get("require_any") and not any(k in ks for k in w["require_any"]):
        raise SystemExit(f"pmc_summary: workload {tag} needs one of {w['require_any']}; found {sorted(ks)}")
    for k in w["forbid"]:
        if k in ks:
            raise SystemExit(f"pmc_summary: workload {tag}: {k} in the window belongs to another config")
    for k in w["once_per_solve"]:
        if k in ks and ks[k]["launches_per_solve"] != 1.0:
            raise SystemExit(f"pmc_summary: workload {tag}: {k} at {ks[k]['launches_per_solve']} "
                             "launches per solve (a window of another config's solves)")


def main():
    fd, wd, sd, outp, tag = sys.argv[1:6]
    window = sys.argv[6] if len(sys.argv) > 6 else "20"
    window = "first" if window == "first" else int(window)
    nsolve = 1 if window == "first" else window
    if tag not in WORKLOADS:
        raise SystemExit(f"pmc_summary: unknown workload {tag}; one of {sorted(WORKLOADS)}")
    fetch, meta, inst = per_kernel(fd, "FETCH_SIZE", window)
    write, _, _ = per_kernel(wd, "WRITE_SIZE", window)
    trows = _rows(sd, "*kernel_trace.csv")
    w0, w1 = _window(trows, window)
    times = {}
    for r in trows:
        if not (w0 < int(r["Dispatch_Id"]) <= w1):
            continue
        times.setdefault(short(r["Kernel_Name"]), []).append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    wl = WORKLOADS[tag]
    res = {"workload": tag + ("_iter0" if window == "first" else ""),  # (bench.py reads PH windows)
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) + "
                     "--kernel-trace --stats of the bench command",
           "fetch_correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section)",
           "scenarios_per_rank": wl["scenarios_per_rank"], "crops_multiplier": wl["crops_multiplier"],
           "window": ("launches of the process's first solve call (Iter0)" if window == "first" else
                      f"launches of the last {window} solve calls (after the "
                      f"{window + 1}-th last summary_kernel dispatch)"),
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        fk, nf = fetch.get(k, (None, 0))
        wk, _ = write.get(k, (None, 0))
        t = times.get(k, [])
        hbm = raw = None
        if fk is not None and wk is not None:
            hbm = round((2.0 * fk + wk) * 1024.0)
            raw = round((fk + wk) * 1024.0)
        res["kernels"][k] = {"instances": sorted(inst.get(k, [])),
                             "fetch_kB_raw": fk, "write_kB": wk, "hbm_bytes_per_launch": hbm,
                             "hbm_bytes_per_launch_uncorrected": raw,
                             "launches_per_solve": round(nf / nsolve, 3),
                             "mean_ns": (sum(t) / len(t)) if t else None, **meta.get(k, {})}
    validate(tag, res, inst)
    with open(outp, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
