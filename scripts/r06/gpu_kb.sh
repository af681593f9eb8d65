#!/bin/bash
# Timing probe: x3_gemm256_af_kernel with k-blocked operand addressing (wrong
# values, same bytes) vs row-major, priced launch at 128^3; the waterfall-free
# descriptors (libm3d.so) vs the previous build (libm3d_old.so) on both priced
# GEMMs; L2->L1 request counters; a parity subset on the new build.
set -o pipefail
OUT=gpurun_out/${1:-r06kb}
mkdir -p $OUT
export TMPDIR=/tmp
leg() {  # lib leg
  timeout -k 10 120 env M3D_LIB_FILE=$1 python -u scripts/kernels_for_pmc.py $2 128 > $OUT/k.json 2> $OUT/k.err || { tail -20 $OUT/k.err; return 1; }
  python3 -c "
import ast; d = ast.literal_eval(open('$OUT/k.json').read().strip().splitlines()[-1]); print('$1 $2', d['avg_launch_ms'], 'ms', d['achieved'], 'TF/s', d['frac'])" | tee -a $OUT/summary.txt
}
step() {  # lib
  timeout -k 10 240 env M3D_LIB_FILE=$1 python -u bench.py --steps 20 --warmup 3 --no-extras --slab-size 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; return 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$1 step', d['ms_per_step'], 'ms (graph)', 'eager', d.get('eager_ms_per_step'))" | tee -a $OUT/summary.txt
}
for rep in 1 2; do
  for lib in libm3d_old.so libm3d_nosk.so libm3d.so; do leg $lib wgrad || exit 1; done
  for lib in libm3d_old.so libm3d.so libm3d_kb1.so libm3d_kb2.so libm3d_kb3.so; do leg $lib gemm || exit 1; done
done
for lib in libm3d_old.so libm3d.so libm3d_old.so libm3d.so; do step $lib || exit 1; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_roi_nms.py tests/test_gpu_conv.py tests/test_gpu_configs.py tests/test_gpu_determinism.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
for lib in libm3d_old.so libm3d_kb3.so; do
  timeout -s KILL 90 env M3D_LIB_FILE=$lib rocprofv3 -f csv --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace -d $OUT/p_$lib -o run -- python3 scripts/kernels_for_pmc.py gemm 128 > $OUT/p_$lib.log 2>&1 || { tail -20 $OUT/p_$lib.log; exit 1; }
done
python3 - <<'PY' | tee -a gpurun_out/r06kb/summary.txt
import csv, glob, collections
for lib in ("libm3d_old.so", "libm3d_kb3.so"):
    fs = glob.glob(f"gpurun_out/r06kb/p_{lib}/**/*counter_collection.csv", recursive=True)
    if not fs: print(lib, "no csv"); continue
    by = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(fs[0])):
        if "x3_gemm256_af_kernel" in r.get("Kernel_Name", ""):
            by[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    d = sorted(by, key=int)[-1]
    print(lib, dict(by[d]))
PY
