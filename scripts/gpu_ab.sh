#!/bin/bash
# A/B of a kernel switch: GPU tests matching EXPR, then the priced leg and a
# short bench per env setting.  Usage: gpurun -- bash scripts/gpu_ab.sh TAG "EXPR" LEG "ENV_A" "ENV_B" ...
set -o pipefail
TAG=$1; EXPR=$2; LEG=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$EXPR" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "$EXPR" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -n 2 $OUT/pytest.log
fi
for envs in "$@"; do
  echo "== $envs"
  env $envs timeout -k 10 120 python -u scripts/kernels_for_pmc.py $LEG 128 > $OUT/leg.txt 2>&1 || { tail -20 $OUT/leg.txt; exit 1; }
  python3 -c "
import ast; d = ast.literal_eval(open('$OUT/leg.txt').read().strip().splitlines()[-1])
print('  leg', d['avg_launch_ms'], 'ms', d['achieved'], 'TF', d['frac'])"
  [ -n "$NOBENCH" ] && continue
  env $envs timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('  step', d['ms_per_step'], 'ms', d['value'], 'vol/s')"
done
echo DONE
