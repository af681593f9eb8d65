#!/bin/bash
# PyramidROIAlign forward timing probes (libm3d_rd1: no output stores, rd2: no corner loads)
set -o pipefail
OUT=gpurun_out/${1:-roiprobe}
mkdir -p $OUT
export TMPDIR=/tmp
for lib in libm3d.so libm3d_rd1.so libm3d_rd2.so; do
  M3D_LIB_FILE=$lib timeout -k 10 200 python -u scripts/roi_ab.py > $OUT/ab.json 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/ab.json').read().strip().splitlines()[-1])
print('$lib', ' '.join(f\"{k}:{v['ms']}ms\" for k, v in d.items() if k != 'mode'))"
done
