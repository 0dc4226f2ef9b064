#!/bin/bash
# HBM traffic of the grouped LF kernel at scale (tools/probe_rank.py, 2^19
# pairs): FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes, per
# MI355X_MICROARCH.md (bytes = 2*1024*FETCH_SIZE + 1024*WRITE_SIZE on gfx950).
# usage: tools/pmc_rank.sh <outdir>
set -euo pipefail
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "k_lf_group" --output-format csv \
      -d "$OUT/raw_$C" -o run -- python3 tools/probe_rank.py --rows-log2 19 --patterns 1024 \
      > "$OUT/rank_$C.log" 2>&1
  find "$OUT/raw_$C" -name "*counter_collection.csv" -exec cp {} "$OUT/counters_$C.csv" \;
  rm -rf "$OUT/raw_$C"
done
python3 - "$OUT" <<'PY'
import csv, json, sys, os
out = sys.argv[1]
def per(c):
    v = {}
    for r in csv.DictReader(open(os.path.join(out, f"counters_{c}.csv"))):
        if "k_lf_group" in r.get("Kernel_Name", "") and r.get("Counter_Name") == c:
            d = int(r["Dispatch_Id"]); v[d] = v.get(d, 0.0) + float(r["Counter_Value"])
    return [v[k] for k in sorted(v)]
f, w = per("FETCH_SIZE"), per("WRITE_SIZE")
res = {"dispatches": [len(f), len(w)], "fetch_bytes": [2 * 1024 * x for x in f], "write_bytes": [1024 * x for x in w]}
json.dump(res, open(os.path.join(out, "pmc_rank.json"), "w"), indent=1)
print(json.dumps(res))
PY
