"""Dispatch sequence of the LAST training step in a rocprofv3 kernel trace (a
serialized trace, bench.py --wgrad-inline, reads as the layer order): one line
per dispatch with its duration, grid and kernel name, plus totals per kernel
name.  Usage: trace_seq.py run_kernel_trace.csv[.gz] [min_us]"""
import csv
import gzip
import sys

f = sys.argv[1]
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
rows = list(csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)))
ends = [int(r["End_Timestamp"]) for r in rows if "sgd_update_kernel" in r["Kernel_Name"]]
lo, hi = ends[-2], ends[-1]
sel = sorted((r for r in rows if int(r["Start_Timestamp"]) >= lo and int(r["End_Timestamp"]) <= hi),
             key=lambda r: int(r["Start_Timestamp"]))
tot = {}
for r in sel:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    name = r["Kernel_Name"]
    short = name.split("(")[0].replace("void ", "").replace("m3d::", "")[:70]
    tot[short] = tot.get(short, 0.0) + d
    if d >= min_us:
        g = "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
        print(f"{(int(r['Start_Timestamp']) - lo) / 1e3:9.1f} {d:8.1f} us  {g:>20s}  {short}")
print(f"--- step window {(hi - lo) / 1e6:.2f} ms, {len(sel)} dispatches, busy {sum(tot.values()) / 1e3:.2f} ms")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:30]:
    print(f"{v / 1e3:8.3f} ms  {k}")
