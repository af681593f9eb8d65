#!/bin/bash
# Effective clock and MFMA busy of the dominant kernel's priced launch and of the
# Winograd point GEMM (MI355X_MICROARCH.md 'DVFS give-back': clock = GRBM_GUI_ACTIVE / 8 / wall).
set -o pipefail
OUT=gpurun_out/${1:-r05clock}
mkdir -p $OUT
export TMPDIR=/tmp
for leg in wgrad gemm; do
  timeout -s KILL 120 rocprofv3 -f csv --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace -d $OUT/c_$leg -o run -- python3 scripts/kernels_for_pmc.py $leg 128 > $OUT/c_$leg.log 2>&1 || { tail -20 $OUT/c_$leg.log; exit 1; }
  rm -f $OUT/c_$leg/run_kernel_trace.csv
done
python3 - <<'PY'
import csv, glob, collections
for leg, kern in (("wgrad", "x3_wgrad_tr_kernel"), ("gemm", "x3_gemm256_af_kernel")):
    f = glob.glob(f"gpurun_out/r05clock/c_{leg}/**/*counter_collection.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if kern in r.get("Kernel_Name", "")]
    by = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        by[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        by[r["Dispatch_Id"]]["_ns"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) if "End_Timestamp" in r else 0
    last = sorted(by, key=int)[-3:]
    for d in last:
        c = by[d]
        ns = c["_ns"]
        clk = c["GRBM_GUI_ACTIVE"] / 8 / ns if ns else float("nan")
        print(leg, kern, "dispatch", d, f"wall {ns/1e3:.1f} us", f"eff clock {clk:.2f} GHz",
              f"MFMA busy / GUI_ACTIVE-per-XCD {c['SQ_VALU_MFMA_BUSY_CYCLES'] / max(c['GRBM_GUI_ACTIVE'] / 8, 1):.1f}")
PY
