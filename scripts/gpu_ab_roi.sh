#!/bin/bash
# A/B of a ROIAlign-forward env switch: the ROI parity tests, then
# the 7^3 / 14^3 legs at 128^3 and 256^3 per env setting.
# Usage: gpurun -- bash scripts/gpu_ab_roi.sh TAG "ENV_A" "ENV_B" ...   (tests run under every ENV but the first)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for envs in "${@:2}"; do
  env $envs timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_roi_nms.py tests/test_gpu_configs.py -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  echo "$envs: $(tail -n 1 $OUT/pytest.log)"
done
for rep in 1 2; do
for envs in "$@"; do
  for S in 128 256; do
    env $envs timeout -k 10 200 python -u - $S > $OUT/leg.txt 2>&1 <<'PY' || { tail -20 $OUT/leg.txt; exit 1; }
import sys
sys.path[:0] = [".", "3d-mask-r-cnn_amd"]
import torch
import bench
from m3d.config import synthetic_rpn_config
from m3d.model import RPN, synthetic_volume
S = int(sys.argv[1])
model = RPN(synthetic_rpn_config(S), device=torch.device("cuda"), seed=1)
with torch.no_grad():
    fmaps = model.features(synthetic_volume(S).to("cuda"))
torch.cuda.synchronize()
print(bench.time_roi_align(fmaps, S, n_rois=128 if S == 128 else 512, reps=5, pools=(7, 14), hi=128 if S == 128 else S))
PY
    python3 -c "
import ast; d = ast.literal_eval(open('$OUT/leg.txt').read().strip().splitlines()[-1])
for k, v in d.items(): print('$envs S=$S', k, v['ms'], 'ms frac', v['frac_hbm'], 'per-roi', v.get('frac_hbm_per_roi'))"
  done
done
done
