#!/bin/bash
# bf16-split stem forward + phased slab Winograd: conv / slab-halo / model / slab tests, then the stem A/B
set -o pipefail
OUT=gpurun_out/r03j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_slab_halo.py tests/test_gpu_model.py -m gpu > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for e in "M3D_STEM_X3=1" "M3D_STEM_X3=0" "M3D_STEM_X3=1"; do
  env $e timeout -k 10 200 python -u scripts/stem_ab.py > $OUT/stem.json 2> $OUT/stem.err || { tail -20 $OUT/stem.err; exit 1; }
  echo "$e $(tail -n 1 $OUT/stem.json)"
done
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread tests/test_gpu_slab.py -m gpu > $OUT/slab.log 2>&1 || { tail -40 $OUT/slab.log; exit 1; }
grep -E "passed|failed" $OUT/slab.log | tail -3
