#!/bin/bash
# A/B of a kernel env switch on the conv layer table + bench step.  Usage: gpu_ab.sh TAG VAR VAL_A VAL_B
set -o pipefail
TAG=$1; VAR=$2; A=$3; B=$4
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for v in $A $B; do
  env $VAR=$v timeout -k 10 300 python3 scripts/conv_bench.py > $OUT/conv_$v.txt 2>&1 || { tail -20 $OUT/conv_$v.txt; exit 1; }
  env $VAR=$v timeout -k 10 300 python3 bench.py --no-extras --slab-size 0 > $OUT/bench_$v.json 2>$OUT/bench_$v.err || { tail -20 $OUT/bench_$v.err; exit 1; }
  env $VAR=$v timeout -k 10 120 python3 -c "import bench, json; print(json.dumps(bench.time_dominant_kernel(128)))" > $OUT/gemm_$v.json 2>&1 || exit 1
  echo "== $VAR=$v"; cat $OUT/conv_$v.txt; cat $OUT/bench_$v.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('step ms', d['ms_per_step'], 'vol/s', d['value'])"; cat $OUT/gemm_$v.json
done
