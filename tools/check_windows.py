"""Measurement check: for every workload the bench line
reports a `traffic` for, the per-kernel times of the committed PMC summary's
window against the HIP-event times of the same kernels in the bench line
run under the profiler (profiles/<round>/<w>_line_under_rocprof.json):
ratio and whether they agree within 10 %.

    python tools/check_windows.py profiles/r04
"""
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "profiles/r04"


def load(name):
    with open(os.path.join(d, name)) as f:
        return json.load(f)


rows = []
f2 = load("f2_line_under_rocprof.json")
k2 = load("pmc_summary_f2.json")["kernels"]
for kname, v in f2["roofline"]["kernels"].items():
    if kname in k2 and v["ms"]:
        rows.append(("F2", kname, v["ms"] * 1e3, k2[kname]["mean_ns"] / 1e3))
f3 = load("f3_line_under_rocprof.json")["f3"]["roofline"]
k3 = load("pmc_summary_f3.json")["kernels"]
for kname, ms in f3["kernel_ms"].items():
    rows.append(("F3", kname, ms * 1e3, k3[kname]["mean_ns"] / 1e3))
f4 = load("f4_line_under_rocprof.json")["f4"]["roofline"]
k4 = load("pmc_summary_f4.json")["kernels"]
phase = sum(k4[k]["mean_ns"] for k in ("big_kernel", "big_team_kernel") if k in k4) / 1e3
rows.append(("F4", "PDHG phase (big_kernel + big_team_kernel)", f4["kernel_ms"] / f4["launches"] * 1e3, phase))
rows.append(("F4", "big_polish_kernel", f4["polish_ms"] / f4["polish_launches"] * 1e3,
             k4["big_polish_kernel"]["mean_ns"] / 1e3))
out = []
for w, k, ev, pmc in rows:
    r = pmc / ev if ev else None
    out.append({"workload": w, "kernel": k, "hip_event_us": round(ev, 2), "pmc_window_us": round(pmc, 2),
                "ratio": round(r, 3) if r else None, "within_10pct": bool(r and abs(r - 1) <= 0.10)})
    print(f"{w:4s} {k:45s} events {ev:10.1f} us  pmc window {pmc:10.1f} us  ratio {r:6.3f}")
json.dump(out, open(os.path.join(d, "window_check.json"), "w"), indent=1)
