#!/bin/bash
# x3_gemm_kernel timing probes on the priced shape: full / no-MFMA / no-loads builds.
set -o pipefail
L=3d-mask-r-cnn_amd/m3d
cp $L/libm3d.so /tmp/libm3d_full.so
for v in full dbg1 dbg2; do
  if [ $v != full ]; then cp $L/libm3d_$v.so $L/libm3d.so; fi
  timeout -k 10 120 python3 -c "
import sys; sys.path[:0]=['.','3d-mask-r-cnn_amd']
import bench
r=bench.time_dominant_kernel(128)
print('$v', r['avg_launch_ms'], 'ms', r['achieved'], 'TF')" 2>&1 | grep -v amdgpu.ids || exit 1
done
cp /tmp/libm3d_full.so $L/libm3d.so
