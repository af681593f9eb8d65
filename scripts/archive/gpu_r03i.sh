#!/bin/bash
# stem weight-gradient kernel: conv / determinism / slab-halo tests, then the stem A/B
set -o pipefail
OUT=gpurun_out/r03i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_slab_halo.py tests/test_gpu_determinism.py -m gpu > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for e in "M3D_STEM_WGRAD=1" "M3D_STEM_WGRAD=0"; do
  env $e timeout -k 10 200 python -u scripts/stem_ab.py > $OUT/stem.json 2> $OUT/stem.err || { tail -20 $OUT/stem.err; exit 1; }
  echo "$e $(tail -n 1 $OUT/stem.json)"
done
