"""Per-kernel HBM bytes per launch from rocprofv3 PMC passes of bench.py.

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR STATS_DIR OUT.json SCENS_PER_RANK CROPS [WINDOW]

FETCH_DIR / WRITE_DIR: `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
output directories (separate passes, csv).  FETCH_SIZE and WRITE_SIZE are in
kB per dispatch; per MI355X_MICROARCH.md (HBM section) FETCH_SIZE on gfx950
reports half the bytes of coalesced reads, so it is doubled here.
STATS_DIR: the `--kernel-trace --stats` run (kernel time per launch).

Window: the launches after the (WINDOW+1)-th last `summary_kernel` dispatch,
i.e. the last WINDOW solve calls (one summary kernel closes each solve) --
with --tol-run 0 and the F3 companion off (or on its own run) these are the
eagerly launched PH iterations whose HIP-event times give the bench line's
`achieved`, so traffic and algorithmic bytes describe the same launches.
Kernels are named by their function name (template arguments dropped);
`launches_per_solve` = launches in the window / WINDOW.  VGPR count and
scratch (spill) bytes per lane come from the same records.
"""
import csv
import glob
import json
import os
import re
import sys

_NAME = re.compile(r"::(\w+)\s*[<(]")


def short(name):
    m = _NAME.search(name)
    if m:
        return m.group(1)
    return name.split("(")[0].strip()


def _rows(d, pattern):
    f = glob.glob(os.path.join(d, pattern))[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def _window_start(rows, window):
    """Dispatch id after which the last `window` solve calls start."""
    summ = [int(r["Dispatch_Id"]) for r in rows if short(r["Kernel_Name"]) == "summary_kernel"]
    summ = sorted(set(summ))
    if len(summ) <= window:
        return -1
    return summ[-window - 1]


def per_kernel(d, counter, window):
    rows = [r for r in _rows(d, "*counter_collection.csv") if r["Counter_Name"] == counter]
    w0 = _window_start(rows, window)
    vals, meta = {}, {}
    for r in rows:
        if int(r["Dispatch_Id"]) <= w0:
            continue
        k = short(r["Kernel_Name"])
        vals.setdefault(k, []).append(float(r["Counter_Value"]))
        meta[k] = {"vgpr": int(r["VGPR_Count"]), "accum_vgpr": int(r["Accum_VGPR_Count"]),
                   "scratch_bytes_per_lane": int(r["Scratch_Size"]),
                   "lds_bytes": int(r["LDS_Block_Size"]), "workgroup": int(r["Workgroup_Size"])}
    return {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}, meta


def main():
    fd, wd, sd, outp, spr, crops = sys.argv[1:7]
    window = int(sys.argv[7]) if len(sys.argv) > 7 else 20
    fetch, meta = per_kernel(fd, "FETCH_SIZE", window)
    write, _ = per_kernel(wd, "WRITE_SIZE", window)
    trows = _rows(sd, "*kernel_trace.csv")
    w0 = _window_start(trows, window)
    times = {}
    for r in trows:
        if int(r["Dispatch_Id"]) <= w0:
            continue
        times.setdefault(short(r["Kernel_Name"]), []).append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) + "
                     "--kernel-trace --stats of the bench command",
           "fetch_correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section)",
           "scenarios_per_rank": int(spr), "crops_multiplier": int(crops),
           "window": f"launches of the last {window} solve calls (after the "
                     f"{window + 1}-th last summary_kernel dispatch)",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        fk, nf = fetch.get(k, (None, 0))
        wk, _ = write.get(k, (None, 0))
        t = times.get(k, [])
        hbm = None
        if fk is not None and wk is not None:
            hbm = round((2.0 * fk + wk) * 1024.0)
        res["kernels"][k] = {"fetch_kB_raw": fk, "write_kB": wk, "hbm_bytes_per_launch": hbm,
                             "launches_per_solve": round(nf / window, 3),
                             "mean_ns": (sum(t) / len(t)) if t else None, **meta.get(k, {})}
    with open(outp, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
