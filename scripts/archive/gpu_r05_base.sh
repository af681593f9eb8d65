#!/bin/bash
# Round-5 baseline: the GPU suite, then per-layer conv table (each conv alone) and serialized
# kernel traces (weight gradients in line) of the 128^3 and 256^3 steps.
# Usage: gpurun -- bash scripts/archive/gpu_r05_base.sh TAG
set -o pipefail
TAG=${1:-r05base}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -n 2 $OUT/pytest_gpu.log
timeout -k 10 240 python scripts/conv_layers.py --size 128 > $OUT/layers128.txt 2>&1 || { tail -20 $OUT/layers128.txt; exit 1; }
echo layers128 done
timeout -k 10 300 rocprofv3 -f csv --kernel-trace -d $OUT/t128 -o run -- python3 bench.py --wgrad-inline --steps 2 --warmup 2 --no-extras --slab-size 0 --size 128 > $OUT/t128.log 2>&1 || { tail -30 $OUT/t128.log; exit 1; }
gzip -f $OUT/t128/run_kernel_trace.csv
echo trace128 done
timeout -k 10 400 rocprofv3 -f csv --kernel-trace -d $OUT/t256 -o run -- python3 bench.py --wgrad-inline --steps 2 --warmup 1 --no-extras --slab-size 0 --size 256 > $OUT/t256.log 2>&1 || { tail -30 $OUT/t256.log; exit 1; }
gzip -f $OUT/t256/run_kernel_trace.csv
echo trace256 done
timeout -k 10 300 rocprofv3 --stats --kernel-trace -d $OUT/inf -o run -- python3 scripts/infer_prof.py --size 256 --reps 5 > $OUT/inf.log 2>&1 || { tail -30 $OUT/inf.log; exit 1; }
python3 scripts/prof_summary.py $OUT/inf/run_kernel_stats.csv 6 40 > $OUT/infer_kernels_256.txt
gzip -f $OUT/inf/run_kernel_trace.csv
echo infer done
