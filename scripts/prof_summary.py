"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels, per-step ms."""
import csv, sys
path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.2f} ms/step {float(r['Percentage']):6.2f}% n={int(r['Calls'])/steps:7.1f} avg={float(r['AverageNs'])/1e3:9.1f}us {r['Name'][:100]}")
print(f"total kernel time {tot/1e6/steps:.2f} ms/step")
