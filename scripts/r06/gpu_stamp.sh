#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r06stamp}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 env M3D_LIB_FILE=libm3d_stamp.so python -u scripts/r06/stamp_gemm.py 128 > $OUT/stamp128.txt 2>&1 || { tail -20 $OUT/stamp128.txt; exit 1; }
cat $OUT/stamp128.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_conv.py tests/test_gpu_configs.py tests/test_gpu_config0.py tests/test_gpu_slab.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
