#!/bin/bash
# Kernel trace of a few bench steps (kept, gzipped) + timeline of the last step.
# Usage: gpurun -- bash scripts/gpu_trace.sh TAG [S] [extra env]
set -o pipefail
TAG=${1:-trace}; S=${2:-128}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 -f csv --kernel-trace -d $OUT/t -o run -- python3 bench.py --steps 3 --warmup 2 --no-extras --slab-size 0 --size $S > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
gzip -f $OUT/t/run_kernel_trace.csv
python3 scripts/trace_timeline.py $OUT/t/run_kernel_trace.csv.gz > $OUT/timeline.txt
python3 scripts/trace_phases.py $OUT/t/run_kernel_trace.csv.gz > $OUT/phases.txt
cat $OUT/timeline.txt $OUT/phases.txt
