set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/w2p; mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -oE "^[[:space:]]*(SQ_|TCC_|TCP_|TA_)[A-Z0-9_]+" $O/counters.txt | sort -u | tr -d ' ' > $O/names.txt || true
wc -l $O/names.txt
P="rocprofv3 -f csv --kernel-trace"
timeout -s KILL 120 $P --pmc FETCH_SIZE -d $O/f -o run -- python3 scripts/kernels_for_pmc.py wgrad 128 > $O/f.log 2>&1 || { tail $O/f.log; exit 1; }
timeout -s KILL 120 $P --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES -d $O/s -o run -- python3 scripts/kernels_for_pmc.py wgrad 128 > $O/s.log 2>&1 || { tail $O/s.log; exit 1; }
timeout -s KILL 120 $P --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD -d $O/s2 -o run -- python3 scripts/kernels_for_pmc.py wgrad 128 > $O/s2.log 2>&1 || { tail $O/s2.log; }
for d in f s s2; do python3 - $O/$d/run_counter_collection.csv <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    if "wgrad_tr" in r.get("Kernel_Name", ""):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k, "n=%d" % len(v), "mean=%.4g" % (sum(v) / len(v)))
PY
done
