set -o pipefail
OUT=gpurun_out/${1:-st}
mkdir -p $OUT
export TMPDIR=/tmp
P="rocprofv3 -f csv"
timeout -s KILL 300 $P --pmc FETCH_SIZE --kernel-trace -d $OUT/f -o run -- python3 bench.py --steps 3 --warmup 1 --eager --no-extras --slab-size 0 > $OUT/f.log 2>&1 || { tail -20 $OUT/f.log; exit 1; }
timeout -s KILL 300 $P --pmc WRITE_SIZE --kernel-trace -d $OUT/w -o run -- python3 bench.py --steps 3 --warmup 1 --eager --no-extras --slab-size 0 > $OUT/w.log 2>&1 || { tail -20 $OUT/w.log; exit 1; }
python3 scripts/step_traffic.py $OUT/f $OUT/w 4 45 > $OUT/step_traffic.txt
rm -f $OUT/f/run_kernel_trace.csv $OUT/w/run_kernel_trace.csv $OUT/f/run_counter_collection.csv $OUT/w/run_counter_collection.csv
