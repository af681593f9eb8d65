#!/bin/bash
# kept-U weight gradient: slab tests, then the bench step + 256^3 depth slab (memory, time)
set -o pipefail
OUT=gpurun_out/r03m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread tests/test_gpu_slab.py tests/test_gpu_slab_halo.py -m gpu > $OUT/slab.log 2>&1 || { tail -40 $OUT/slab.log; exit 1; }
grep -E "passed|failed" $OUT/slab.log | tail -2
timeout -k 10 400 python -u bench.py --no-extras > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1])
print('step', d['ms_per_step'], d['value'], 'slab', d['depth_slab']['ms_per_step'], d['depth_slab'].get('peak_mem_gb'))"
