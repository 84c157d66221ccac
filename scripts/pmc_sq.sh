#!/bin/bash
# One rocprofv3 --pmc pass (no trace domains, graphs off) over a bench command, summarised
# per kernel name into $OUT/summary.json. Counters (at most 8 SQ + 4 TCC per pass; FETCH_SIZE
# takes 3 TCC): $COUNTERS. SQ wave counters are quad-cycles summed over waves; the
# fractions are shares of the summed wave lifetime (SQ_WAVE_CYCLES):
#   wait_any      parked on s_waitcnt / barrier
#   wait_inst_any stalled at instruction issue (dependency / pipe busy)
#   active_inst   issuing
# FETCH_SIZE is doubled on gfx950 (it counts half of a 16 B/lane stream: MI355X_MICROARCH.md).
# Usage: OUT=gpurun_out/pmc_pp COUNTERS="..." KFILTER="k_mmq4|k_fa" bash scripts/pmc_sq.sh <cmd...>
cd "$(dirname "$0")/.."
ROOTDIR=$PWD
OUT=${OUT:-gpurun_out/pmc_sq}
COUNTERS=${COUNTERS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$ROOTDIR"
GGML_MI355X_DISABLE_GRAPHS=1 timeout -s KILL ${TMO:-240} rocprofv3 --pmc $COUNTERS -d $OUT/raw -o pmc --output-format csv -- "$@" \
  > $OUT/run.log 2>&1 || { echo "pmc pass failed"; tail -20 $OUT/run.log; exit 1; }
python3 - "$OUT" "${KFILTER:-.}" <<'PY'
import csv, glob, json, os, re, sys
out, kf = sys.argv[1], re.compile(sys.argv[2])
f = glob.glob(os.path.join(out, "raw", "**", "*counter_collection.csv"), recursive=True)[0]
per = {}   # kernel -> dispatch -> counter -> value
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if not kf.search(k):
        continue
    k = k.split("(")[0]
    d = per.setdefault(k, {}).setdefault(r["Dispatch_Id"], {})
    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
res = {}
for k, ds in per.items():
    tot = {}
    for d in ds.values():
        for c, v in d.items():
            tot[c] = tot.get(c, 0.0) + v
    n = len(ds)
    avg = {c: v / n for c, v in tot.items()}
    e = {"dispatches": n, "per_dispatch": avg}
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        for c, name in (("SQ_WAIT_ANY", "wait_any_frac"), ("SQ_WAIT_INST_ANY", "wait_inst_any_frac"),
                        ("SQ_ACTIVE_INST_ANY", "active_inst_frac")):
            if c in avg:
                e[name] = round(avg[c] / wc, 3)
    if "SQ_LDS_BANK_CONFLICT" in avg and avg.get("SQ_ACTIVE_INST_LDS"):
        e["lds_bank_conflict_frac"] = round(avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_ACTIVE_INST_LDS"], 3)
    # MFMA pipe utilisation: busy cycles (summed over SIMDs) over 1,024 SIMDs x the kernel's
    # cycles (GRBM_GUI_ACTIVE is summed over the 8 XCDs: MI355X_MICROARCH.md, DVFS give-back)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and avg.get("GRBM_GUI_ACTIVE"):
        e["mfma_util"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * avg["GRBM_GUI_ACTIVE"] / 8), 3)
    if "FETCH_SIZE" in avg:
        e["hbm_read_bytes"] = int(2 * avg["FETCH_SIZE"] * 1024)
    res[k] = e
json.dump({"counters": sorted({c for k in per.values() for d in k.values() for c in d}), "kernels": res},
          open(os.path.join(out, "summary.json"), "w"), indent=1)
for k, e in sorted(res.items(), key=lambda x: -x[1]["dispatches"]):
    print(k[:70], {x: y for x, y in e.items() if x != "per_dispatch"})
PY
