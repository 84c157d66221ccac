#!/bin/bash
# HBM traffic of the roofline kernel (bench.py's SwiGLU GEMV cycle) from rocprofv3 PMC
# counters, one counter per pass (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950),
# no trace domains besides the kernel trace. gfx950 FETCH_SIZE counts half the bytes of a
# 16 B/lane streaming read (MI355X_MICROARCH.md §HBM): traffic = 2*FETCH + WRITE (KiB).
cd "$(dirname "$0")/.."
ROOTDIR=$PWD
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$ROOTDIR"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${TMO:-600} rocprofv3 --pmc $c -d $OUT/$c -o pmc --output-format csv -- \
    python3 bench.py --roofline-only > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; tail -20 $OUT/$c.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys
out = sys.argv[1]
def per_dispatch(counter):
    f = glob.glob(os.path.join(out, counter, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = {}
    for r in csv.DictReader(open(f)):
        if "k_gemv2" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.setdefault(r["Dispatch_Id"], 0.0)
            vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = sorted(vals.values())
    return v[len(v) // 4:] or v          # drop warm-up dispatches
fetch, write = per_dispatch("FETCH_SIZE"), per_dispatch("WRITE_SIZE")
roof = json.loads([l for l in open(os.path.join(out, "FETCH_SIZE.log")) if l.startswith("{")][-1])
fk, wk = sum(fetch) / len(fetch), sum(write) / len(write)
rec = {"kernel": roof["kernel"], "bytes_per_launch": roof["bytes_per_launch"],
       "fetch_size_kib": fk, "write_size_kib": wk, "dispatches": len(fetch),
       "hbm_bytes_per_launch": int((2 * fk + wk) * 1024),
       "note": "FETCH_SIZE doubled (gfx950 counts half of a 16 B/lane stream), WRITE_SIZE as is; separate --pmc passes"}
print(json.dumps(rec))
json.dump(rec, open(os.path.join(out, "pmc_glu.json"), "w"), indent=1)
PY
