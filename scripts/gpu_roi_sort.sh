#!/bin/bash
# PyramidROIAlign forward variants at configs[2]/[3] shapes (scripts/roi_ab.py), each env twice.
# Usage: gpurun -- bash scripts/gpu_roi_sort.sh TAG "ENV_A" "ENV_B" ...
set -o pipefail
OUT=gpurun_out/${1:-roisort}; shift
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for envs in "$@"; do
  env $envs timeout -k 10 200 python -u scripts/roi_ab.py > $OUT/ab.json 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/ab.json').read().strip().splitlines()[-1])
print('$envs', ' '.join(f\"{k}:{v['ms']}ms/{v['frac_hbm']}/{v['sha'][:6]}\" for k, v in d.items() if k != 'mode'))"
done
done
