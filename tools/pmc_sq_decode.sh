#!/bin/bash
# SQ wave-state counters of the fused decode kernel over the default bench
# (eager replay, so each timed step is its own dispatch): one rocprofv3 --pmc
# pass of 8 SQ counters (the SQ block's limit), summarised per dispatch for
# the last --steps k_decode<false, true, 1024> launches.
# usage: tools/pmc_sq_decode.sh <outdir> [bench args...]
set -euo pipefail
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
trap 'rm -rf "$OUT/raw"' EXIT
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --kernel-include-regex "k_decode" --output-format csv \
    -d "$OUT/raw" -o run -- python3 bench.py --no-cpu --no-c4 --no-gather --eager-replay "$@" \
    > "$OUT/bench.json" 2> "$OUT/bench.log"
F=$(find "$OUT/raw" -name "*counter_collection.csv" | head -1)
cp "$F" "$OUT/counters_sq.csv"
python3 - "$OUT/counters_sq.csv" "$OUT/sq_summary.json" <<'PY'
import csv, json, sys
rows = {}
for r in csv.DictReader(open(sys.argv[1])):
    if "k_decode<false, true, 1024>" not in r.get("Kernel_Name", ""):
        continue
    d = rows.setdefault(int(r["Dispatch_Id"]), {})
    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
last = [rows[k] for k in sorted(rows)][-20:]
tot = {c: sum(d.get(c, 0.0) for d in last) for c in last[0]} if last else {}
res = {"source": "rocprofv3 --pmc SQ_* over bench.py --eager-replay, last 20 k_decode<false, true, 1024> dispatches",
       "dispatches": len(last), "totals": tot}
if tot:
    res["wait_any_frac"] = tot["SQ_WAIT_ANY"] / tot["SQ_WAVE_CYCLES"]
    res["wait_inst_any_frac"] = tot["SQ_WAIT_INST_ANY"] / tot["SQ_WAVE_CYCLES"]
    res["active_inst_frac"] = tot["SQ_ACTIVE_INST_ANY"] / tot["SQ_WAVE_CYCLES"]
    res["valu_per_wave"] = tot["SQ_INSTS_VALU"] / tot["SQ_WAVES"]
    res["vmem_wr_per_wave"] = tot["SQ_INSTS_VMEM_WR"] / tot["SQ_WAVES"]
    res["vmem_rd_per_wave"] = tot["SQ_INSTS_VMEM_RD"] / tot["SQ_WAVES"]
print(json.dumps(res, indent=1))
json.dump(res, open(sys.argv[2], "w"), indent=1)
PY
