#!/bin/bash
# Prefetching NMS reduction (nms_reduce_pf_kernel): the NMS / ProposalLayer GPU
# tests, then bench.time_nms at the training shapes with M3D_NMS_REDUCE=1 / 0.
set -o pipefail
OUT=gpurun_out/nmspf
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_roi_nms.py tests/test_gpu_configs.py -k "nms or proposal" > $OUT/pytest.log 2>&1 \
    || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for v in 1 0; do
  M3D_NMS_REDUCE=$v timeout -k 10 120 python -u - <<'PY' || exit 1
import os, sys, json
sys.path[:0] = [".", "3d-mask-r-cnn_amd"]
import torch, bench
dev = torch.device("cuda:0")
for k, mo, thr in ((10000, 3000, 0.9), (15000, 6000, 0.7), (15000, 6000, 0.3), (4000, 4000, 0.5)):
    r = bench.time_nms(dev, k=k, max_out=mo, thr=thr, reps=10)
    print("M3D_NMS_REDUCE=" + os.environ["M3D_NMS_REDUCE"], json.dumps(r))
PY
done
