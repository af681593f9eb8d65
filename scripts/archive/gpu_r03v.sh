#!/bin/bash
# Fused RPN losses + ProposalLayer launched after the backward: GPU tests, then
# the 128^3 step A/B of both switches.
set -o pipefail
OUT=gpurun_out/r03v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_rpn_loss.py tests/test_gpu_model.py tests/test_gpu_dp.py > $OUT/pytest.log 2>&1 \
    || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
bash scripts/gpu_step_ab.sh r03v_ab "M3D_FUSED_RPN_LOSS=1 M3D_PROPOSALS_AFTER_BWD=1" \
    "M3D_FUSED_RPN_LOSS=0 M3D_PROPOSALS_AFTER_BWD=0" "M3D_FUSED_RPN_LOSS=1 M3D_PROPOSALS_AFTER_BWD=0" \
    "M3D_FUSED_RPN_LOSS=0 M3D_PROPOSALS_AFTER_BWD=1"
