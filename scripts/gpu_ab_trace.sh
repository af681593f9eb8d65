#!/bin/bash
# A/B by kernel time: one-step serial kernel trace (M3D_WGRAD_STREAM=0, no
# proposals) per variant; prints GPU busy time of the step and the top kernels.
# Usage: VARIANTS='"A=1" "A=2"' bash scripts/gpu_ab_trace.sh
set -o pipefail
O=gpurun_out/abt; mkdir -p $O
export TMPDIR=/tmp
i=0
eval "set -- $VARIANTS"
for v in "$@"; do
  i=$((i+1))
  env $v M3D_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 -f csv --kernel-trace -d $O/t$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-extras --no-proposals > $O/log$i 2>&1 || { tail -20 $O/log$i; exit 1; }
  echo "== $v"
  python3 scripts/trace_timeline.py $O/t$i/run_kernel_trace.csv | sed -n 1,4p
  python3 - $O/t$i/run_kernel_trace.csv <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
ends = [int(r["End_Timestamp"]) for r in rows if "sgd_update_kernel" in r["Kernel_Name"]]
lo, hi = ends[-2], ends[-1]
agg = collections.defaultdict(float)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s >= lo and e <= hi:
        agg[r["Kernel_Name"].split("(")[0].split("<")[0][-28:]] += (e - s) / 1e6
print("  " + "; ".join(f"{k.strip()} {v:.2f}" for k, v in sorted(agg.items(), key=lambda x: -x[1])[:8]))
PY
  rm -rf $O/t$i
done
