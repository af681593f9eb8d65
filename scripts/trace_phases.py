"""Critical-path view of the LAST training step in a rocprofv3 kernel trace:
per queue, the busy time and the idle time between consecutive kernels of that
queue, split at the first backward kernel of the compute queue (the queue that
runs the stem conv).  Usage: trace_phases.py run_kernel_trace.csv[.gz]"""
import csv
import gzip
import sys

f = sys.argv[1]
rows = list(csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)))
ends = [int(r["End_Timestamp"]) for r in rows if "sgd_update_kernel" in r["Kernel_Name"]]
lo, hi = ends[-2], ends[-1]
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"])
            for r in rows if int(r["Start_Timestamp"]) >= lo and int(r["End_Timestamp"]) <= hi)
main_q = ks[0][2]
bwd_keys = ("bwd", "wgrad", "wino_grad", "dgrad", "sgd_")
first_bwd = next(s for s, e, q, n in ks if q == main_q and any(k in n for k in bwd_keys))
print(f"step {(hi - lo) / 1e6:.2f} ms; compute queue {main_q}; forward {(first_bwd - ks[0][0]) / 1e6:.2f} ms, "
      f"backward+update {(hi - first_bwd) / 1e6:.2f} ms")
for q in sorted({k[2] for k in ks}):
    qs = [k for k in ks if k[2] == q]
    for name, a, b in (("fwd", lo, first_bwd), ("bwd", first_bwd, hi)):
        sel = [k for k in qs if a <= k[0] < b]
        if not sel:
            continue
        busy = sum(e - s for s, e, _, _ in sel)
        idle = sum(max(0, sel[i + 1][0] - sel[i][1]) for i in range(len(sel) - 1))
        print(f"  queue {q} {name}: {len(sel):4d} kernels, busy {busy / 1e6:6.2f} ms, idle between {idle / 1e6:6.2f} ms")
        agg = {}
        for s, e, _, n in sel:
            key = n.split("(")[0][-60:]
            agg[key] = agg.get(key, 0) + e - s
        for key, t in sorted(agg.items(), key=lambda x: -x[1])[:8]:
            print(f"      {t / 1e6:6.2f} ms  {key}")
