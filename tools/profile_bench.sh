#!/bin/bash
# rocprofv3 kernel-trace + stats of one bench run (GPU box).  Keeps only the
# stats CSVs (the full per-dispatch trace can exceed gpurun's 64 MiB merge cap).
# usage: tools/profile_bench.sh <outdir> [bench args...]
set -euo pipefail
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/raw" -o run -- python3 bench.py --no-cpu "$@" > "$OUT/bench.json" 2> "$OUT/bench.log"
find "$OUT/raw" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/raw"
