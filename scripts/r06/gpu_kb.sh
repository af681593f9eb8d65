#!/bin/bash
# Timing probe: x3_gemm256_af_kernel with k-blocked operand addressing (wrong
# values, same bytes) vs row-major, priced launch at 128^3; plus L2->L1 request
# counters for the base and the both-blocked build.
set -o pipefail
OUT=gpurun_out/${1:-r06kb}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for lib in libm3d.so libm3d_kb1.so libm3d_kb2.so libm3d_kb3.so; do
  timeout -k 10 120 env M3D_LIB_FILE=$lib python -u scripts/kernels_for_pmc.py gemm 128 > $OUT/k.json 2> $OUT/k.err || { tail -20 $OUT/k.err; exit 1; }
  python3 -c "
import ast; d = ast.literal_eval(open('$OUT/k.json').read().strip().splitlines()[-1]); print('$lib gemm', d['avg_launch_ms'], 'ms', d['achieved'], 'TF/s', d['frac'])" | tee -a $OUT/summary.txt
done
done
for lib in libm3d.so libm3d_kb3.so; do
  timeout -s KILL 90 env M3D_LIB_FILE=$lib rocprofv3 -f csv --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum --kernel-trace -d $OUT/p_$lib -o run -- python3 scripts/kernels_for_pmc.py gemm 128 > $OUT/p_$lib.log 2>&1 || { tail -20 $OUT/p_$lib.log; exit 1; }
done
python3 - <<'PY' | tee -a gpurun_out/r06kb/summary.txt
import csv, glob, collections
for lib in ("libm3d.so", "libm3d_kb3.so"):
    fs = glob.glob(f"gpurun_out/r06kb/p_{lib}/**/*counter_collection.csv", recursive=True)
    if not fs: print(lib, "no csv"); continue
    by = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(fs[0])):
        if "x3_gemm256_af_kernel" in r.get("Kernel_Name", ""):
            by[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    d = sorted(by, key=int)[-1]
    print(lib, dict(by[d]))
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_roi_nms.py tests/test_gpu_conv.py tests/test_gpu_configs.py tests/test_gpu_determinism.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
