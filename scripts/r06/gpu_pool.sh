#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r06pool}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_slab_halo.py -m gpu -x -q -k "maxpool" --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 120 python -u scripts/r06/pool_time.py 256 | tee $OUT/pool_time.txt
