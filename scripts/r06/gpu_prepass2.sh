#!/bin/bash
# data-gradient pre-pass at every size (forward's from 128^3): tests, then
# same-box A/B (nn.WINO_V_PREPASS 0 / 1) at 64^3 and 128^3 and the configs[0] leg.
set -o pipefail
OUT=gpurun_out/${1:-r06pre2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wino_prepass.py tests/test_gpu_determinism.py tests/test_gpu_config0.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
grep -c PASSED $OUT/tests.log
step() {
  timeout -k 10 240 python -u scripts/bench_ab.py $1 -- --steps 20 --warmup 3 --size $2 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; return 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$1 $2 step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
}
for rep in 1 2; do for spec in nn.WINO_V_PREPASS=0 nn.WINO_V_PREPASS=1; do step $spec 64 || exit 1; step $spec 128 || exit 1; done; done
for spec in nn.WINO_V_PREPASS=0 nn.WINO_V_PREPASS=1; do
  timeout -k 10 300 env M3D_AB_SPEC=$spec python -u - > $OUT/c0.txt 2>&1 <<'PY' || { tail -20 $OUT/c0.txt; exit 1; }
import importlib, os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "3d-mask-r-cnn_amd")]
from m3d import nn as mnn
k, v = os.environ["M3D_AB_SPEC"].split("=")
setattr(mnn, k.split(".")[1], bool(int(v)))
import torch, bench
r = bench.configs0_leg(torch.device("cuda"), 10, 3) if hasattr(bench, "configs0_leg") else None
print("c0", r["ms_per_step"] if r else None, r.get("eager_ms_per_step") if r else None)
PY
  echo "$spec $(tail -1 $OUT/c0.txt)" | tee -a $OUT/summary.txt
done
