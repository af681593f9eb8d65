#!/bin/bash
# X3 vs f32: winofwd leg per-kernel times, GPU conv tests under X3, bench
# ms/step alternating modes (3 runs each, noise).
set -o pipefail
O=gpurun_out/x3ab; mkdir -p $O
export TMPDIR=/tmp
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 -f csv --kernel-trace -d $O/$tag -o run -- python3 scripts/kernels_for_pmc.py winofwd 128 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  python3 - $O/$tag/run_kernel_trace.csv $tag <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    agg[r["Kernel_Name"].split("(")[0][-60:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(sys.argv[2], "; ".join(f"{k.split('::')[-1]} {sum(v[1:])/max(1,len(v)-1):.0f}us" for k, v in agg.items() if "gemm" in k or "wino" in k or "x3" in k))
PY
  rm -rf $O/$tag
}
M3D_GEMM_X3=1 timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or wino" > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
run f32 M3D_GEMM_X3=0
run x3 M3D_GEMM_X3=1
for i in 1 2 3; do for x in 0 1; do
  M3D_GEMM_X3=$x timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-extras > $O/b 2>&1 || { tail -5 $O/b; exit 1; }
  echo "x3=$x $(grep -o '"ms_per_step": [0-9.]*' $O/b)"
done; done
