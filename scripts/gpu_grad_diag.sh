#!/bin/bash
set -o pipefail
for cfg in "2 2" "4 2" "4 4"; do
  set -- $cfg
  M3D_WINO_NZ=$1 M3D_WINO_DGRAD_NZ=$2 timeout -k 10 200 python3 scripts/grad_err_diag.py 2>&1 | grep "median" || exit 1
done
for cfg in "4 2" "4 4"; do
  set -- $cfg
  M3D_WINO_NZ=$1 M3D_WINO_DGRAD_NZ=$2 timeout -k 10 300 python3 bench.py --no-extras --slab-size 0 > /tmp/b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('/tmp/b.json')); print('NZ=$1 DGRAD=$2 step ms', d['ms_per_step'], 'vol/s', d['value'])"
done
