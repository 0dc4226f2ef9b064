#!/bin/bash
# rocprofv3 kernel-trace + stats of one bench run (GPU box).  Keeps the stats
# CSV and a summary of the fused decode kernel's dispatches (all, and the last
# --steps ones = the timed graph replay); the full per-dispatch trace can
# exceed gpurun's 64 MiB merge cap, so it is dropped.
# usage: tools/profile_bench.sh <outdir> [bench args...]
set -euo pipefail
OUT=$1; shift
mkdir -p "$OUT"
# the raw trace can exceed gpurun's merge cap: never leave it behind
trap 'rm -rf "$OUT/raw"' EXIT
export TMPDIR=/tmp
rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/raw" -o run -- python3 bench.py --no-cpu --no-c4 "$@" > "$OUT/bench.json" 2> "$OUT/bench.log"
find "$OUT/raw" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
TRACE=$(find "$OUT/raw" -name "*kernel_trace.csv" | head -1)
python3 - "$TRACE" "$OUT/decode_dispatches.json" "$@" <<'PY'
import csv, json, sys
trace, out, args = sys.argv[1], sys.argv[2], sys.argv[3:]
steps = int(args[args.index("--steps") + 1]) if "--steps" in args else 20
d = []
with open(trace) as f:
    for r in csv.DictReader(f):
        if "k_decode<false, true," in r.get("Kernel_Name", ""):  # <PACKED, DO_LF, threads>
            d.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
d.sort()
if not d:
    sys.exit("no k_decode<false, true, *> dispatches in " + trace)
dur = [x[1] / 1e3 for x in d]
t = dur[-steps:]
res = {"kernel": "k_decode<false, true, *>", "dispatches": len(dur), "avg_us_all": sum(dur) / len(dur),
       "timed_dispatches": len(t), "avg_us_timed": sum(t) / len(t), "min_us_timed": min(t), "max_us_timed": max(t),
       "note": "timed = the last --steps dispatches (the bench's timed graph replay); all includes warmup, "
               "the three replays used for the step estimate and the standalone mask-only graphs' k_decode<false,false> excluded"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
PY
# the sharded rehearsal's kernels (bench's C4 leg at N = 1): per-shard packed decode, the OR pass
python3 tools/trace_durations.py "$TRACE" "k_decode<true, true," --out "$OUT/c4_shard_decode_dispatches.json" > /dev/null || true
python3 tools/trace_durations.py "$TRACE" "k_or_unpack" --out "$OUT/c4_or_dispatches.json" || true
python3 tools/trace_durations.py "$TRACE" "k_lf_group" --out "$OUT/lf_group_dispatches.json" > /dev/null || true
# the rank legs (2^19 / 2^21 pairs: the in-wave sweep, by grid size) against the bench's events
python3 tools/trace_durations.py "$TRACE" "k_lf_sweep" --out "$OUT/lf_sweep_dispatches.json" > /dev/null || true
rm -rf "$OUT/raw"
