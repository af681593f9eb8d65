#!/bin/bash
# rocprofv3 kernel stats of the bench step, then per priced launch separate
# FETCH_SIZE / WRITE_SIZE PMC passes (kernel-trace only, never with sys/runtime
# trace).  Usage (repo root): gpurun --timeout 1200 -- bash scripts/gpu_prof.sh TAG [S]
set -o pipefail
TAG=${1:-r01}
S=${2:-128}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P="rocprofv3 -f csv"
STEPS=5; WARM=2
timeout -k 10 400 $P --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --eager --steps $STEPS --warmup $WARM --no-extras --size $S > $OUT/prof_bench.log 2>&1 || { echo "rocprof bench failed"; tail -30 $OUT/prof_bench.log; exit 1; }
python3 scripts/prof_summary.py $OUT/prof/run_kernel_stats.csv $((STEPS + WARM)) 40 > $OUT/bench_kernels.txt
rm -f $OUT/prof/run_kernel_trace.csv
NR=$([ "$S" = 128 ] && echo 128 || echo 512)
LEGS=${LEGS:-"gemm:x3_gemm256_af_kernel:wino_gemm_x3af_rpn_shared1_S$S wgrad:x3_wgrad:wino_wgrad_gemm_rpn_shared1_S$S direct:conv_gemm_kernel:direct_conv_rpn_shared1_S$S roi7:line_fwd_sl_kernel:pyramid_fwd_pool7_S${S}_N$NR roi14:line_fwd_sl_kernel:pyramid_fwd_pool14_S${S}_N$NR"}
for spec in $LEGS; do
  IFS=: read leg kern key <<< "$spec"
  timeout -k 10 300 $P --kernel-trace --stats -d $OUT/k_$leg -o run -- python3 scripts/kernels_for_pmc.py $leg $S > $OUT/k_$leg.log 2>&1 || { echo "rocprof $leg failed"; tail -30 $OUT/k_$leg.log; exit 1; }
  timeout -k 10 300 $P --pmc FETCH_SIZE --kernel-trace -d $OUT/f_$leg -o run -- python3 scripts/kernels_for_pmc.py $leg $S > $OUT/f_$leg.log 2>&1 || { echo "pmc fetch $leg failed"; tail -30 $OUT/f_$leg.log; exit 1; }
  timeout -k 10 300 $P --pmc WRITE_SIZE --kernel-trace -d $OUT/w_$leg -o run -- python3 scripts/kernels_for_pmc.py $leg $S > $OUT/w_$leg.log 2>&1 || { echo "pmc write $leg failed"; tail -30 $OUT/w_$leg.log; exit 1; }
  python3 scripts/pmc_traffic.py $OUT/f_$leg/run_counter_collection.csv $OUT/w_$leg/run_counter_collection.csv $kern ${key} $OUT/traffic.json 3 || exit 1
  python3 scripts/prof_summary.py $OUT/k_$leg/run_kernel_stats.csv 1 8 > $OUT/k_$leg.txt
  rm -f $OUT/?_$leg/run_kernel_trace.csv
done
cat $OUT/bench_kernels.txt $OUT/k_*.txt $OUT/traffic.json
echo DONE
