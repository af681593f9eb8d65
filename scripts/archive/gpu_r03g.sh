#!/bin/bash
# Round-3 re-entry check: kernel trace + per-phase timeline of the 128^3 step on
# the current tree, and the step with the weight gradients in line (no side stream).
set -o pipefail
OUT=gpurun_out/r03g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 -f csv --kernel-trace --stats -d $OUT/t -o run -- python3 bench.py --steps 3 --warmup 2 --no-extras --slab-size 0 > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
python3 scripts/prof_summary.py $OUT/t/run_kernel_stats.csv 5 45 > $OUT/kernels.txt
gzip -f $OUT/t/run_kernel_trace.csv
python3 scripts/trace_phases.py $OUT/t/run_kernel_trace.csv.gz > $OUT/phases.txt
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b1.json 2> $OUT/b1.err || { tail -20 $OUT/b1.err; exit 1; }
M3D_WGRAD_STREAM=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b0.json 2> $OUT/b0.err || { tail -20 $OUT/b0.err; exit 1; }
cat $OUT/phases.txt; head -30 $OUT/kernels.txt
python3 -c "
import json
for f in ('b1','b0'):
    d=json.loads(open('$OUT/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['ms_per_step'])"
