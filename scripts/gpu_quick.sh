#!/bin/bash
# quick perf check: gpu tests (optional -k), conv layer table, bench step, dominant GEMM
set -o pipefail
TAG=$1; KEXPR=$2
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "$KEXPR" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
timeout -k 10 300 python3 scripts/conv_bench.py > $OUT/conv.txt 2>&1 || { tail -20 $OUT/conv.txt; exit 1; }
timeout -k 10 300 python3 bench.py --no-extras --slab-size 0 > $OUT/bench.json 2>$OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 120 python3 -c "import bench, json; print(json.dumps(bench.time_dominant_kernel(128)))" > $OUT/gemm.json 2>&1 || exit 1
grep -v amdgpu.ids $OUT/conv.txt; python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('step ms', d['ms_per_step'], 'vol/s', d['value'])"; grep achieved $OUT/gemm.json | cut -c1-200
