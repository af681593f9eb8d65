#!/bin/bash
# A/B of the batched (Winograd) GEMM launch modes: M3D_GEMM_PERSIST x M3D_GEMM_NBUF
set -o pipefail
mkdir -p gpurun_out/gab
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "wino or gemm or conv" > gpurun_out/gab/pytest.log 2>&1 || { tail -30 gpurun_out/gab/pytest.log; exit 1; }
tail -1 gpurun_out/gab/pytest.log
for cfg in "0 1" "1 1" "1 2" "0 2"; do
  set -- $cfg
  M3D_GEMM_PERSIST=$1 M3D_GEMM_NBUF=$2 timeout -k 10 120 python3 -c "
import sys; sys.path[:0]=['.','3d-mask-r-cnn_amd']
import bench, json
r = bench.time_dominant_kernel(128, reps=10)
print('persist=$1 nbuf=$2', r['achieved'], r['frac'], r['avg_launch_ms'])" 2>&1 | grep persist || exit 1
done
