#!/bin/bash
# Step-time A/B of env settings (bench --no-extras, N=1, 128^3), each run twice.
# Usage: gpurun -- bash scripts/gpu_step_ab.sh TAG "ENV_A" "ENV_B" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for envs in "$@"; do
  env $envs timeout -k 10 ${TMO:-200} python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-extras --slab-size 0 --size ${S:-128} > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$envs', 'step', d['ms_per_step'], 'ms', d['value'], 'vol/s')"
done
done
grep "priority" $OUT/b.err | head -2 || true
