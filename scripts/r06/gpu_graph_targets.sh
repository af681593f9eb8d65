#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r06gt}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_targets.py tests/test_gpu_determinism.py tests/test_gpu_config0.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 400 python -u scripts/r06/legs.py > $OUT/legs.txt 2> $OUT/legs.err || { tail -30 $OUT/legs.err; exit 1; }
cat $OUT/legs.txt
