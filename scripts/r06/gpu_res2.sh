#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r06res2}
mkdir -p $OUT
export TMPDIR=/tmp
P=res2a_branch2b+res2b_branch2b+res2c_branch2b
timeout -k 10 500 python -u scripts/r06/slab_ab.py - $P > $OUT/slab.txt 2> $OUT/slab.err || { tail -20 $OUT/slab.err; exit 1; }
cat $OUT/slab.txt
timeout -k 10 500 python -u scripts/r06/grad_policy.py $P tests/test_gpu_configs.py -m gpu -x -q -s -k "gradients" --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/grad.log 2>&1; echo "grad rc=$?"
grep "gradients:" $OUT/grad.log | cut -c1-260
