"""Timeline of the LAST training step in a rocprofv3 kernel trace (window =
between the last two sgd_update_kernel dispatches): wall, busy time per
queue, union busy time, and the largest idle gaps (no kernel on any queue).
Usage: trace_timeline.py run_kernel_trace.csv[.gz]"""
import csv
import gzip
import sys

f = sys.argv[1]
rows = list(csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)))
ends = [int(r["End_Timestamp"]) for r in rows if "sgd_update_kernel" in r["Kernel_Name"]]
lo, hi = ends[-2], ends[-1]
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"])
             for r in rows if int(r["Start_Timestamp"]) >= lo and int(r["End_Timestamp"]) <= hi))
print(f"step window {(hi - lo) / 1e6:.2f} ms, {len(ks)} dispatches")
per_q = {}
for s, e, q, _ in ks:
    per_q[q] = per_q.get(q, 0) + (e - s)
for q, t in sorted(per_q.items()):
    print(f"  queue {q}: busy {t / 1e6:.2f} ms")
busy, cur_s, cur_e, gaps, prev_name = 0, None, None, [], ""
for s, e, q, n in ks:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev_name[:60], n[:60]))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev_name = n if e >= (cur_e or 0) else prev_name
busy += cur_e - cur_s
print(f"  union busy {busy / 1e6:.2f} ms, idle {(hi - lo - busy) / 1e6:.2f} ms in {len(gaps)} gaps")
for g, a, b in sorted(gaps, reverse=True)[:15]:
    print(f"    gap {g / 1e3:8.1f} us after {a} -> {b}")
