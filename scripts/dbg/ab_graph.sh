set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/abg; mkdir -p $OUT
for rep in 1 2; do
for g in "" "--graph"; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 $g > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('graph=$g', d['ms_per_step'], 'ms', d['value'])"
done
done
