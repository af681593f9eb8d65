#!/bin/bash
# Kernel trace of the 128^3 step on the current tree: compute-queue idle gaps.
set -o pipefail
OUT=gpurun_out/r03w
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 -f csv --kernel-trace -d $OUT/t -o run -- python3 bench.py --steps 3 --warmup 2 --no-extras --slab-size 0 > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
gzip -f $OUT/t/run_kernel_trace.csv
python3 scripts/trace_gaps.py $OUT/t/run_kernel_trace.csv.gz 40 > $OUT/gaps.txt
python3 scripts/trace_phases.py $OUT/t/run_kernel_trace.csv.gz > $OUT/phases.txt
cat $OUT/gaps.txt
