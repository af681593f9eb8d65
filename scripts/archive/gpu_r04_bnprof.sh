#!/bin/bash
# rocprofv3 kernel stats of the 128^3 step with the fused BN backward off / on
# (same box): which kernels gained / lost time.
set -o pipefail
OUT=gpurun_out/${1:-r04_bnprof}
mkdir -p $OUT
export TMPDIR=/tmp
for f in 0 1; do
  M3D_BN_FUSE=$f timeout -k 10 400 rocprofv3 -f csv --kernel-trace --stats -d $OUT/p$f -o run -- python3 bench.py --steps 5 --warmup 2 --no-extras --slab-size 0 > $OUT/b$f.log 2>&1 || { echo "rocprof $f failed"; tail -30 $OUT/b$f.log; exit 1; }
  python3 scripts/prof_summary.py $OUT/p$f/run_kernel_stats.csv 7 40 > $OUT/k$f.txt
  rm -f $OUT/p$f/run_kernel_trace.csv
done
head -45 $OUT/k0.txt $OUT/k1.txt
