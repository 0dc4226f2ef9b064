#!/bin/bash
# (round 5: FMIDX_EPI_CHUNKS is a compile-time variant now -- make ... VFLAGS=-DFMIDX_EPI_CHUNKS=2)
# Epilogue chunks per thread (FMIDX_EPI_CHUNKS), one process each:
# tools/bench_epilogue.py lines per variant into $1.
set -uo pipefail
OUT=${1:-gpurun_out/epi}
mkdir -p "$OUT"
for v in 1 2 4; do
  echo "[epi] chunks $v $(date +%T)"
  FMIDX_EPI_CHUNKS=$v timeout -k 10 120 python -u tools/bench_epilogue.py > "$OUT/epi_c$v.jsonl" 2> "$OUT/epi_c$v.log" || exit $?
  cat "$OUT/epi_c$v.jsonl"
done
