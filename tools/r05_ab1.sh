#!/bin/bash
# Round-5 A/B: early zero-fill pacing (s_sleep between a thread's zero stores)
# against the default, then cold phase stamps of the default kernel.
set -euo pipefail
O=gpurun_out/r05_ab1
mkdir -p "$O"
L=fm-index-constrained-decoding_amd/fmidx
timeout -k 10 600 python -u tools/ab_decode.py --reps 7 $L/libfmidx.so $L/libfmidx_ez8.so $L/libfmidx_ez16.so \
    $L/libfmidx_ez32.so $L/libfmidx.so > "$O/ab.jsonl" 2> "$O/ab.log"
cat "$O/ab.jsonl"
COLD=1 QUIET=1 timeout -k 10 300 python -u tools/probe_stamps.py > "$O/stamps_cold.log" 2>&1
grep -E "^step|SUMMARY" "$O/stamps_cold.log" | head -30
echo "r05_ab1 done"
