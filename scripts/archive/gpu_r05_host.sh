#!/bin/bash
# Gradient parity of the configs[1] step (median printed), the new fused /
# batched paths' tests, the host enqueue profile of the 128^3 step
# (scripts/host_overhead.py: enqueue vs wall per step and a cProfile of the
# enqueue) and the per-layer conv table at 256^3.
# Usage: gpurun -- bash scripts/archive/gpu_r05_host.sh TAG
set -o pipefail
TAG=${1:-r05host}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_configs.py tests/test_gpu_bnfuse.py tests/test_gpu_conv.py -k "config1_gradients or fused or bn_affine or conv1_x3" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
grep -E "gradients:|passed|failed" $OUT/pytest.log | cut -c1-300
timeout -k 10 300 python -u scripts/host_overhead.py > $OUT/host_overhead.txt 2>&1 || { tail -30 $OUT/host_overhead.txt; exit 1; }
grep "host enqueue\|synchronising" $OUT/host_overhead.txt
timeout -k 10 500 python -u scripts/conv_layers.py --size 256 --reps 3 > $OUT/layers256.txt 2>&1 || { tail -20 $OUT/layers256.txt; exit 1; }
tail -1 $OUT/layers256.txt
