#!/bin/bash
# HBM traffic of the LF launch at scale (the in-wave sweep from 2^19 rows) (tools/probe_rank.py, 2^19
# pairs) and of one grouped launch per LF path class (--by-path): FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 passes, per MI355X_MICROARCH.md (bytes =
# 2*1024*FETCH_SIZE + 1024*WRITE_SIZE on gfx950).
# usage: tools/pmc_rank.sh <outdir>
set -euo pipefail
OUT=$1
mkdir -p "$OUT"
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "k_lf_group|k_lf_sweep" --output-format csv \
      -d "$OUT/raw_$C" -o run -- python3 tools/probe_rank.py --rows-log2 19 --patterns 1024 --by-path \
      --out "$OUT/probe_$C.json" > "$OUT/rank_$C.log" 2>&1
  find "$OUT/raw_$C" -name "*counter_collection.csv" -exec cp {} "$OUT/counters_$C.csv" \;
  rm -rf "$OUT/raw_$C"
done
python3 - "$OUT" <<'PY'
import csv, json, sys, os
sys.path.insert(0, os.path.join(os.getcwd(), "tools"))
from pmc_summarize import lib_sha16
out = sys.argv[1]
def per(c):
    v = {}
    for r in csv.DictReader(open(os.path.join(out, f"counters_{c}.csv"))):
        if ("k_lf_group" in r.get("Kernel_Name", "") or "k_lf_sweep" in r.get("Kernel_Name", "")) and r.get("Counter_Name") == c:
            d = int(r["Dispatch_Id"]); v[d] = v.get(d, 0.0) + float(r["Counter_Value"])
    return [v[k] for k in sorted(v)]
f, w = per("FETCH_SIZE"), per("WRITE_SIZE")
probe = json.load(open(os.path.join(out, "probe_FETCH_SIZE.json")))
paths = probe.get("by_path", [])
k = len(paths)
by = []
for e, fb, wb in zip(paths, f[-k:] if k else [], w[-k:] if k else []):
    fetch, write = 2 * 1024 * fb, 1024 * wb
    by.append(dict(e, fetch_bytes=fetch, write_bytes=write,
                   fetch_per_alg_byte=(fetch / e["alg_bytes"]) if e["alg_bytes"] else None,
                   fetch_per_row=fetch / max(1, e["rows"])))
big = f[:-k] if k else f
res = {"lib_sha16": lib_sha16(), "dispatches": [len(f), len(w)],
       "fetch_bytes": [2 * 1024 * x for x in big], "write_bytes": [1024 * x for x in (w[:-k] if k else w)],
       "by_path": by}
json.dump(res, open(os.path.join(out, "pmc_rank.json"), "w"), indent=1)
print(json.dumps(res))
PY
