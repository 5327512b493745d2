"""Summarise tools/fetch_calib under rocprofv3 (measurement tool): per access
pattern the known bytes, FETCH_SIZE / WRITE_SIZE (kB per dispatch) and their
ratio, i.e. the factor that turns the counter into bytes for that pattern.

    python tools/fetch_calib_summary.py FETCH_DIR WRITE_DIR LOG > out.json

LOG holds the program's "CALIB name known_bytes line_bytes" lines (one per
dispatch, in dispatch order; the two profiled runs print them twice).
"""
import csv
import glob
import json
import os
import sys


def rows(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    out = [r for r in csv.DictReader(open(f))
           if r["Counter_Name"] == counter and not r["Kernel_Name"].startswith("__amd_rocclr")]
    out.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [(r["Kernel_Name"], float(r["Counter_Value"])) for r in out]


def main():
    fd, wd, log = sys.argv[1:4]
    known = []
    for ln in open(log):
        p = ln.split()
        if len(p) == 4 and p[0] == "CALIB":
            known.append((p[1], int(p[2]), int(p[3])))
    known = known[:len(known) // 2] if len(known) % 2 == 0 and len(known) > 6 else known[:6]
    fetch = rows(fd, "FETCH_SIZE")
    write = rows(wd, "WRITE_SIZE")
    if len(fetch) != len(known) or len(write) != len(known):
        raise SystemExit(f"fetch_calib_summary: {len(known)} patterns, {len(fetch)} / {len(write)} dispatches")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of tools/fetch_calib "
                     "(a 2 GiB buffer, 8x the Infinity Cache)", "patterns": {}}
    for (name, nb, lb), (kn, fk), (_, wk) in zip(known, fetch, write):
        e = {"kernel": kn, "known_bytes": nb, "FETCH_SIZE_kB": fk, "WRITE_SIZE_kB": wk}
        c = wk if name.startswith("write") else fk
        e["bytes_per_counter_byte"] = round(nb / (c * 1024.0), 4) if c else None
        if lb:
            e["line_bytes_128B"] = lb
            e["line_bytes_per_counter_byte"] = round(lb / (c * 1024.0), 4) if c else None
        res["patterns"][name] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
