#!/bin/bash
# Same-box step A/B of round 5's fusions: the BN-ReLU backward in the split
# GEMM's epilogue (nn.X3_BN_FUSE), the batched BN affine (backbone.BN_AFFINE_BATCHED),
# the 1x1x1 conv epilogue in the split GEMM (build libm3d_noepi.so: M3D_TUNE_CONV1_EPI=0).
set -o pipefail
OUT=gpurun_out/${1:-r05fuse}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # label, lib, switches
  timeout -k 10 240 env M3D_LIB_FILE=$2 python -u scripts/bench_ab.py "$3" -- --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
}
for rep in 1 2; do
  run default libm3d.so ""
  run x3_bn_fuse_off libm3d.so nn.X3_BN_FUSE=0
  run bn_affine_per_layer libm3d.so backbone.BN_AFFINE_BATCHED=0
  run conv1_epi_off libm3d_noepi.so ""
done
