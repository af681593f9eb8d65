"""Per-dispatch view of a rocprofv3 kernel trace: the dispatches of kernels
matching SUBSTR in the LAST `per_step` dispatches of that kernel, with grid
sizes and durations.  Usage: trace_top.py run_kernel_trace.csv SUBSTR [per_step]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
n = int(sys.argv[3]) if len(sys.argv) > 3 else len(rows)
rows = rows[-n:]
tot = 0.0
out = []
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    g = "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
    out.append((d, g, r["Kernel_Name"][:70]))
for d, g, k in sorted(out, reverse=True):
    print(f"{d:9.1f} us  grid {g:>22s}  {k}")
print(f"total {tot / 1e3:.3f} ms over {len(rows)} dispatches")
