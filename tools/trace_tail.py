"""Print the last N kernel dispatches of a rocprofv3 kernel trace (start offset, duration)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
N = int(sys.argv[2]) if len(sys.argv) > 2 else 30
t0 = int(rows[-N]["Start_Timestamp"])
for r in rows[-N:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:60]} grid={r['Grid_Size_X']} wg={r['Workgroup_Size_X']} vgpr={r['VGPR_Count']} agpr={r['Accum_VGPR_Count']} lds={r['LDS_Block_Size']} scr={r['Scratch_Size']}")
