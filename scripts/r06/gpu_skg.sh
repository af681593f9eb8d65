#!/bin/bash
# grouped stream-K (libm3d_skg.so: partner column tiles in lockstep) vs the
# current build: priced wgrad launch times, its PMC FETCH / WRITE bytes, the
# stream-K shape tests, and the 128^3 / 256^3 steps.  bash scripts/r06/gpu_skg.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r06skg}
mkdir -p $OUT
export TMPDIR=/tmp
M3D_LIB_FILE=libm3d_skg.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv.py -k "stream_k or batched_wgrad or wino_weight_gradient" tests/test_gpu_determinism.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
grep -c PASSED $OUT/tests.log
leg() {  # lib leg
  timeout -k 10 120 env M3D_LIB_FILE=$1 python -u scripts/kernels_for_pmc.py $2 128 > $OUT/k.json 2> $OUT/k.err || { tail -20 $OUT/k.err; return 1; }
  python3 -c "
import ast; d = ast.literal_eval(open('$OUT/k.json').read().strip().splitlines()[-1]); print('$1 $2', d['avg_launch_ms'], 'ms', d['achieved'], 'TF/s', d['frac'])" | tee -a $OUT/summary.txt
}
for rep in 1 2; do for lib in libm3d.so libm3d_skg.so; do leg $lib wgrad || exit 1; done; done
for lib in libm3d.so libm3d_skg.so; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 env M3D_LIB_FILE=$lib rocprofv3 -f csv --pmc $c --kernel-trace -d $OUT/p_${lib}_$c -o run -- python3 scripts/kernels_for_pmc.py wgrad 128 > $OUT/p.log 2>&1 || { tail -20 $OUT/p.log; exit 1; }
  done
  python3 scripts/pmc_traffic.py $OUT/p_${lib}_FETCH_SIZE/run_counter_collection.csv $OUT/p_${lib}_WRITE_SIZE/run_counter_collection.csv x3_wgrad wgrad_$lib $OUT/traffic.json 3 > /dev/null || exit 1
done
python3 -c "
import json; d = json.load(open('$OUT/traffic.json')); [print(k, round(v['hbm_bytes_per_launch'] / 1e9, 3), 'GB') for k, v in d.items()]" | tee -a $OUT/summary.txt
step() {
  timeout -k 10 240 env M3D_LIB_FILE=$1 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; return 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$1 step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
}
for rep in 1 2; do for lib in libm3d.so libm3d_skg.so; do step $lib || exit 1; done; done
for lib in libm3d.so libm3d_skg.so; do
  M3D_LIB_FILE=$lib timeout -k 10 400 python -u scripts/r06/mod_ab.py - > $OUT/slab_$lib.txt 2> $OUT/slab.err || { tail -20 $OUT/slab.err; exit 1; }
  echo "$lib 256 $(cat $OUT/slab_$lib.txt | tr '\n' ' ')" | tee -a $OUT/summary.txt
done
