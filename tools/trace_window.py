"""Per-kernel durations and dispatch gaps of F2's bench window from a
rocprofv3 --kernel-trace CSV: the passes 6..25 (update_w_conv dispatches 5..24
of the run, or loop_kernel launches when the persistent path ran).

    python tools/trace_window.py ktr_kernel_trace.csv [first_pass_index] [passes]
"""
import collections
import csv
import sys

f = sys.argv[1]
p0 = int(sys.argv[2]) if len(sys.argv) > 2 else 5
NP = int(sys.argv[3]) if len(sys.argv) > 3 else 20
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))


def nm(r):
    return r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40]


idx = [i for i, r in enumerate(rows) if "active_set" in nm(r)]
seq = rows[idx[p0]:idx[p0 + NP]]
tot = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3
print(f"passes {p0 + 1}..{p0 + NP}: {tot:.1f} us, {tot / NP:.2f} us per pass")
dur = collections.defaultdict(float)
gap = collections.defaultdict(float)
cnt = collections.Counter()
prev = None
for r in seq:
    k = nm(r)
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[k] += (e - s) / 1e3
    cnt[k] += 1
    if prev is not None:
        gap[k] += (s - prev) / 1e3
    prev = e
for k in dur:
    print(f"{k:42s} n {cnt[k]:3d} dur/pass {dur[k] / NP:6.2f} gap-before/pass {gap[k] / NP:6.2f}")
