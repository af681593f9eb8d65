#!/bin/bash
# rocprofv3 kernel stats of the 128^3 step (default build), one pass.
set -o pipefail
OUT=gpurun_out/${1:-r04_prof1}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 -f csv --kernel-trace --stats -d $OUT/p -o run -- python3 bench.py --steps 5 --warmup 2 --no-extras --slab-size 0 --size ${S:-128} > $OUT/b.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/b.log; exit 1; }
python3 scripts/prof_summary.py $OUT/p/run_kernel_stats.csv 7 60 > $OUT/k.txt
python3 scripts/trace_gaps.py $OUT/p/run_kernel_trace.csv 15 > $OUT/gaps.txt 2>&1 || true
python3 scripts/trace_phases.py $OUT/p/run_kernel_trace.csv > $OUT/phases.txt 2>&1 || true
gzip -f $OUT/p/run_kernel_trace.csv
cat $OUT/gaps.txt $OUT/phases.txt
cat $OUT/k.txt
