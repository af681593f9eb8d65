#!/bin/bash
# The full bench line (with step-roofline tables) + host overhead on one box.
# Usage: gpurun --timeout 900 -- bash scripts/archive/gpu_r04_bench.sh TAG
set -o pipefail
TAG=${1:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
M3D_STEP_ROOFLINE_TABLE=$OUT/step_roofline_128.json M3D_STEP_ROOFLINE_TABLE_256=$OUT/step_roofline_256.json \
  timeout -k 10 780 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps(d["summary"]))
for k in ("roofline", "step_roofline", "cpu_baseline", "cpu_ops", "nms", "configs0", "targets_in_step", "deterministic"):
    print(k, json.dumps(d.get(k))[:700])
print("depth_slab", json.dumps({k: v for k, v in d.get("depth_slab", {}).items() if k != "step_roofline"})[:500])
print("slab_roofline", json.dumps(d.get("depth_slab", {}).get("step_roofline"))[:700])
r = d.get("roi_align_256", {})
print("roi256", json.dumps({k: r.get(k) for k in ("pool7", "pool14", "bwd")})[:1200])
PY
echo DONE
