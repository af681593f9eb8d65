#!/bin/bash
# stem forward timing probes (libm3d_sx{1,2,3}.so: no MFMA / no stores / no window fetch)
set -o pipefail
OUT=gpurun_out/${1:-stemprobe}
mkdir -p $OUT
export TMPDIR=/tmp
for lib in libm3d.so libm3d_sx1.so libm3d_sx2.so libm3d_sx3.so; do
  M3D_LIB_FILE=$lib timeout -k 10 200 python -u scripts/stem_ab.py > $OUT/stem.json 2> $OUT/stem.err || { tail -20 $OUT/stem.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/stem.json').read().strip().splitlines()[-1])
print('$lib', {k: v['ms'] for k, v in d.items() if k.startswith('S')})"
done
