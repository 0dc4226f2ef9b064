#!/bin/bash
# HBM traffic of the hot kernel (and the standalone LF kernel) from PMC counters (GPU box), per
# MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE in separate passes
# (TCC slots), kilobytes; on gfx950 FETCH_SIZE counts half the bytes of wide
# coalesced reads, so bytes = 2*1024*FETCH_SIZE + 1024*WRITE_SIZE.
# usage: tools/pmc_traffic.sh <outdir> [bench args...]
set -euo pipefail
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "k_decode|k_lf" --output-format csv \
      -d "$OUT/raw_$C" -o run -- python3 bench.py --no-cpu --no-c4 --eager-replay "$@" \
      > "$OUT/bench_$C.json" 2> "$OUT/bench_$C.log"
  find "$OUT/raw_$C" -name "*counter_collection.csv" -exec cp {} "$OUT/counters_$C.csv" \;
  rm -rf "$OUT/raw_$C"
done
python3 tools/pmc_summarize.py "$OUT" "$@"
