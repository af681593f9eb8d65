#!/bin/bash
# Per-layer data-gradient tile (nn.WINO_DGRAD_Y4): gradient medians of the
# policies (scripts/grad_table.py), then the 128^3 step of each (graph replay).
set -o pipefail
OUT=gpurun_out/${1:-r05tiley}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/grad_table.py --out $OUT/grad.json --variants base,y4_shared1,y4_p2,y4_fpn,y4_all > $OUT/grad.log 2>&1 || { tail -30 $OUT/grad.log; exit 1; }
grep median $OUT/grad.log | cut -c1-200
for sw in nn.WINO_DGRAD_Y4= nn.WINO_DGRAD_Y4=rpn_conv_shared1+fpn_p2 nn.WINO_DGRAD_Y4=rpn_conv_shared1+fpn_p2+fpn_p3+fpn_p4+fpn_p5 "nn.WINO_DGRAD_Y4=*"; do
  timeout -k 10 240 python -u scripts/bench_ab.py "$sw" -- --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$sw', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
done
