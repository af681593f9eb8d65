#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r06c0prof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/p -o run -- python3 scripts/r06/c0_time.py > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
f=$(find $OUT/p -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats.csv
t=$(find $OUT/p -name '*kernel_trace.csv' | head -1); python3 - "$t" <<'PY' > $OUT/timeline.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# last 20 steps of back-to-back replays: take the final 40% of the trace
n = len(rows); tail = rows[int(n * 0.75):]
t0, t1 = int(tail[0]["Start_Timestamp"]), int(tail[-1]["End_Timestamp"])
busy = collections.defaultdict(float); cnt = collections.Counter()
for r in tail:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    k = r["Kernel_Name"][:70]; busy[k] += d; cnt[k] += 1
span = (t1 - t0) / 1e3
print("span_us", round(span), "kernels", len(tail), "sum_us", round(sum(busy.values())))
# union of busy intervals (any stream)
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in tail)
u = 0; cs, ce = iv[0]
for s, e in iv[1:]:
    if s > ce: u += ce - cs; cs, ce = s, e
    else: ce = max(ce, e)
u += ce - cs
print("busy_union_us", round(u / 1e3), "idle_frac", round(1 - u / (t1 - t0), 3))
for k, v in sorted(busy.items(), key=lambda kv: -kv[1])[:30]:
    print(f"{v:10.1f} us {cnt[k]:6d} x {v / cnt[k]:8.1f}  {k}")
PY
cat $OUT/timeline.txt | head -40
