set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/w2c; mkdir -p $O
for dbg in ${DBGS:-0 1 3 5}; do
  M3D_X3W_DBG=$dbg timeout -s KILL 120 rocprofv3 -f csv --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $O/d$dbg -o run -- python3 scripts/kernels_for_pmc.py wgrad 128 > $O/d$dbg.log 2>&1 || { tail $O/d$dbg.log; exit 1; }
  python3 - $O/d$dbg $dbg <<'PY'
import csv, sys, glob, collections
d = sys.argv[1]
rows = list(csv.DictReader(open(d + "/run_counter_collection.csv")))
tr = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr if "wgrad_tr" in r["Kernel_Name"]]
agg = collections.defaultdict(list)
for r in rows:
    if "wgrad_tr" in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
g = sum(agg["GRBM_GUI_ACTIVE"]) / len(agg["GRBM_GUI_ACTIVE"])
t = sum(durs) / len(durs)
print("DBG", sys.argv[2], "dur_us %.1f" % (t / 1e3), "GRBM_GUI_ACTIVE %.4g" % g, "eff_clock_GHz %.3f" % (g / 8 / t))
PY
done
