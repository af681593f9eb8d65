"""Idle gaps of the compute queue inside the LAST training step of a rocprofv3
kernel trace: total idle, the largest gaps with the kernels either side, and
the idle time per forward/backward region (split at the first backward kernel).
Usage: trace_gaps.py run_kernel_trace.csv[.gz] [n_largest]"""
import csv
import gzip
import sys

f = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = list(csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)))
ends = [int(r["End_Timestamp"]) for r in rows if "sgd_update_kernel" in r["Kernel_Name"]]
lo, hi = ends[-2], ends[-1]
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"])
            for r in rows if int(r["Start_Timestamp"]) >= lo and int(r["End_Timestamp"]) <= hi)
main_q = ks[0][2]
q = [k for k in ks if k[2] == main_q]
t0 = q[0][0]
# time when ANY queue is busy (union), to see gaps where the whole GPU idles
iv = sorted((s, e) for s, e, _, _ in ks)
union, cs, ce = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > ce:
        union += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
union += ce - cs
span = hi - lo
print(f"step {span / 1e6:.2f} ms; compute queue {main_q}: {len(q)} kernels; "
      f"GPU busy (any queue) {union / 1e6:.2f} ms, all-idle {(span - union) / 1e6:.2f} ms")
gaps = []
for a, b in zip(q, q[1:]):
    g = b[0] - a[1]
    if g > 0:
        gaps.append((g, (a[1] - t0) / 1e3, a[3].split("(")[0][-45:], b[3].split("(")[0][-45:]))
print(f"compute-queue idle between kernels {sum(g for g, *_ in gaps) / 1e6:.2f} ms")
for g, t, a, b in sorted(gaps, reverse=True)[:n]:
    print(f"  {g / 1e3:7.1f} us at {t:8.1f} us  after {a:45s} before {b}")
