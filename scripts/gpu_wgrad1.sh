#!/bin/bash
# 1x1x1 weight gradients alone at the 128^3 step's shapes: rate per shape, the
# wgrad_tr m-split floor A/B (M3D_X3W_TR_MINM), kernel stats.
set -o pipefail
OUT=gpurun_out/wg1
mkdir -p $OUT
export TMPDIR=/tmp
for v in 64 256 1024; do
  echo "== M3D_X3W_TR_MINM=$v"
  M3D_X3W_TR_MINM=$v timeout -k 10 120 python3 scripts/wgrad1_bench.py > $OUT/w$v.log 2>&1 || { tail -20 $OUT/w$v.log; exit 1; }
  cat $OUT/w$v.log
done
timeout -k 10 120 rocprofv3 -f csv --kernel-trace --stats -d $OUT/p -o run -- python3 scripts/wgrad1_bench.py > $OUT/p.log 2>&1 || { tail -20 $OUT/p.log; exit 1; }
python3 scripts/prof_summary.py $OUT/p/run_kernel_stats.csv 1 12 2>/dev/null || head -12 $OUT/p/run_kernel_stats.csv
