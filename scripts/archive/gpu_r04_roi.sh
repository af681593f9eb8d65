#!/bin/bash
# ROI kernels: parity tests + grad-image / forward timing.  Usage: gpurun -- bash scripts/archive/gpu_r04_roi.sh TAG
set -o pipefail
TAG=${1:-r04roi}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_roi_nms.py tests/test_gpu_configs.py -k "grad_image or pyramid or crop" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/roi_bwd_bench.py > $OUT/roi_bwd.log 2>&1 || { tail -20 $OUT/roi_bwd.log; exit 1; }
cat $OUT/roi_bwd.log
