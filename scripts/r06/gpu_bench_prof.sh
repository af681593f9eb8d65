#!/bin/bash
# the full bench line and, on the same box, rocprofv3 kernel stats of the two
# priced launches (kernels_for_pmc.py gemm / wgrad), so the bench's HIP-event
# launch times and rocprof's averages come from one machine.
set -o pipefail
TAG=${1:-r06bp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
M3D_STEP_ROOFLINE_TABLE=$OUT/step_roofline_128.json M3D_STEP_ROOFLINE_TABLE_256=$OUT/step_roofline_256.json \
  timeout -k 10 1000 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['wgrad_gemm']['avg_launch_ms'], json.dumps(d.get('summary')))"
for leg in gemm wgrad; do
  timeout -k 10 300 rocprofv3 -f csv --kernel-trace --stats -d $OUT/k_$leg -o run -- python3 scripts/kernels_for_pmc.py $leg 128 > $OUT/k_$leg.log 2>&1 || { echo "rocprof $leg failed"; tail -30 $OUT/k_$leg.log; exit 1; }
  python3 scripts/prof_summary.py $OUT/k_$leg/run_kernel_stats.csv 1 6 > $OUT/k_$leg.txt
  rm -f $OUT/k_$leg/run_kernel_trace.csv
  head -2 $OUT/k_$leg.txt
done
