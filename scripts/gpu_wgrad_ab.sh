#!/bin/bash
# A/B of weight-gradient launch parameters (M3D_WGRAD_K64, M3D_WGRAD_MINM): conv tests, step time.
set -o pipefail
O=gpurun_out/wgab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "conv or model" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "1 256" "0 256" "1 512" "1 1024" "1 128"; do
  set -- $cfg
  M3D_WGRAD_K64=$1 M3D_WGRAD_MINM=$2 timeout -k 10 300 python3 bench.py --no-extras --slab-size 0 > $O/b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/b.json')); print('K64=$1 MINM=$2 step ms', d['ms_per_step'])"
done
for k in 1 0; do
  M3D_WGRAD_K64=$k timeout -k 10 300 python3 scripts/conv_bench.py 2>/dev/null | grep -v "^  +wino" | awk -v k=$k '{print "K64=" k, $0}' | grep "1x1\|stem\|TOTAL"
done
