#!/bin/bash
# GPU tests matching EXPR + the full default bench line.  Usage: gpurun -- bash scripts/gpu_quick.sh TAG "EXPR"
set -o pipefail
TAG=$1; EXPR=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "$EXPR" > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 700 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"])
for k in ("roofline", "configs0", "targets_in_step", "cpu_baseline", "roi_align_bwd", "depth_slab", "mrcnn_inference"):
    print(k, json.dumps(d.get(k))[:600])
r = d.get("roi_align_256", {})
print("roi256", json.dumps({k: r.get(k) for k in ("pool7", "pool14", "bwd")})[:900])
PY
