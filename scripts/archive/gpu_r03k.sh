#!/bin/bash
# stem forward variants: conv / slab-halo / model tests (default kernel), then the stem A/B
set -o pipefail
OUT=gpurun_out/r03k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_slab_halo.py tests/test_gpu_model.py -m gpu > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for e in "M3D_STEM_X3=2" "M3D_STEM_X3=0" "M3D_STEM_X3=2"; do
  env $e timeout -k 10 200 python -u scripts/stem_ab.py > $OUT/stem.json 2> $OUT/stem.err || { tail -20 $OUT/stem.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/stem.json').read().strip().splitlines()[-1])
print('$e', {k: (v['ms'], v['rel_err_y']) for k, v in d.items() if k.startswith('S')})"
done
