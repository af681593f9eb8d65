#!/bin/bash
# HIP-graph step vs eager: GPU test, bench alternating (3x), serial traces.
set -o pipefail
O=gpurun_out/gab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k graphed > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
for i in 1 2 3; do for v in "--graph" ""; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-extras $v > $O/b 2>&1 || { tail -5 $O/b; exit 1; }
  echo "graph${v} $(grep -o '"ms_per_step": [0-9.]*' $O/b)"
done; done
for v in "--graph" ""; do
  timeout -k 10 300 rocprofv3 -f csv --kernel-trace -d $O/t -o run -- python3 bench.py --steps 3 --warmup 2 --no-extras $v > $O/tl 2>&1 || { tail -20 $O/tl; exit 1; }
  echo "== trace graph$v"; python3 scripts/trace_timeline.py $O/t/run_kernel_trace.csv | head -8
  rm -rf $O/t
done
