#!/bin/bash
# Serialized kernel trace (weight gradients in line, M3D_WGRAD_STREAM=0) of a
# few 128^3 steps, for per-layer attribution.  Usage: gpurun -- bash scripts/archive/gpu_r04_trace.sh TAG [S]
set -o pipefail
TAG=${1:-r04tr}; S=${2:-128}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export M3D_WGRAD_STREAM=0
timeout -k 10 300 rocprofv3 -f csv --kernel-trace -d $OUT/t -o run -- python3 bench.py --steps 2 --warmup 2 --no-extras --slab-size 0 --size $S > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
gzip -f $OUT/t/run_kernel_trace.csv
ls -la $OUT/t
