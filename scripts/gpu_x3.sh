#!/bin/bash
# X3 (3-way bf16 split) modes vs f32 MFMA: GPU conv/model tests under X3,
# per-kernel trace of one step, bench ms/step for each mode.
set -o pipefail
O=gpurun_out/x3; mkdir -p $O
export TMPDIR=/tmp
MODES=${MODES:-"0 1"}
M3D_GEMM_X3=${TESTMODE:-1} timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or wino or gemm or model" > $O/tests.txt 2>&1; rc=$?
tail -4 $O/tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for x in $MODES; do
  M3D_GEMM_X3=$x M3D_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 -f csv --kernel-trace -d $O/t$x -o run -- python3 bench.py --steps 1 --warmup 1 --no-extras --no-proposals > $O/tlog$x 2>&1 || { tail -20 $O/tlog$x; exit 1; }
  python3 scripts/trace_top.py $O/t$x/run_kernel_trace.csv "gemm_kernel" 300 > $O/gemm$x.txt
  python3 scripts/trace_timeline.py $O/t$x/run_kernel_trace.csv > $O/tl$x.txt 2>&1 || true
  echo "== x3=$x"; head -8 $O/gemm$x.txt; tail -1 $O/gemm$x.txt; head -3 $O/tl$x.txt
  gzip -f $O/t$x/run_kernel_trace.csv
  M3D_GEMM_X3=$x timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-extras > $O/b$x 2>&1 || { tail -5 $O/b$x; exit 1; }
  echo "x3=$x $(grep -o '"ms_per_step": [0-9.]*' $O/b$x)"
done
