#!/bin/bash
# producer/consumer ROIAlign forward: parity tests under it, then the A/B
set -o pipefail
OUT=gpurun_out/${1:-roipc}
mkdir -p $OUT
export TMPDIR=/tmp
M3D_ROI_PC=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_roi_nms.py tests/test_gpu_config3.py "tests/test_gpu_configs.py::test_config2_pyramid_roi_align_and_grad_image" -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash scripts/gpu_roi_sort.sh ${1:-roipc}/ab "M3D_ROI_PC=0" "M3D_ROI_PC=1"
