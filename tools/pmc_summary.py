"""Per-kernel HBM bytes per launch from rocprofv3 PMC passes of bench.py.

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR STATS_DIR OUT.json SCENS_PER_RANK CROPS [WINDOW]

FETCH_DIR / WRITE_DIR: `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
output directories (separate passes, csv).  FETCH_SIZE and WRITE_SIZE are in
kB per dispatch; per MI355X_MICROARCH.md (HBM section) FETCH_SIZE on gfx950
reports half the bytes of coalesced reads, so it is doubled here.
STATS_DIR: the `--kernel-trace --stats` run (kernel time per launch).
Only the last WINDOW launches of each kernel are kept (default 20 = bench.py's
--steps): with --tol-run 0 --hbm-crops 0 they are the eagerly launched PH
iterations whose HIP-event times and polish/PDHG counts give the bench line's
`achieved`, so traffic and algorithmic bytes describe the same launches.
"""
import csv
import glob
import json
import os
import sys

KERNELS = ("active_set_kernel", "polish_kernel", "pdhg_kernel", "summary_kernel",
           "update_w_conv_kernel", "update_w_kernel", "loop_conv_local_kernel")


def short(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def per_kernel(d, counter, window):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    vals = {}
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        if k and r["Counter_Name"] == counter:
            vals.setdefault(k, []).append(float(r["Counter_Value"]))
    out = {}
    for k, v in vals.items():
        v = v[-window:]
        out[k] = sum(v) / len(v) if v else None
    return out


def main():
    fd, wd, sd, outp, spr, crops = sys.argv[1:7]
    window = int(sys.argv[7]) if len(sys.argv) > 7 else 20
    fetch = per_kernel(fd, "FETCH_SIZE", window)
    write = per_kernel(wd, "WRITE_SIZE", window)
    times = {}
    f = glob.glob(os.path.join(sd, "*kernel_trace.csv"))[0]
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        if k:
            times.setdefault(k, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) + "
                     "--kernel-trace --stats of `python bench.py --tol-run 0 --no-cpu-baseline`",
           "fetch_correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section)",
           "scenarios_per_rank": int(spr), "crops_multiplier": int(crops),
           "window": f"last {window} launches of each kernel (the bench's event-timed iterations)",
           "kernels": {}}
    for k in KERNELS:
        if k not in fetch and k not in write:
            continue
        fk = fetch.get(k)
        wk = write.get(k)
        t = times.get(k, [])
        t = t[-window:]
        hbm = None
        if fk is not None and wk is not None:
            hbm = round((2.0 * fk + wk) * 1024.0)
        res["kernels"][k] = {"fetch_kB_raw": fk, "write_kB": wk, "hbm_bytes_per_launch": hbm,
                             "mean_ns": (sum(t) / len(t)) if t else None}
    with open(outp, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
