#!/bin/bash
# Memory-side read requests by size (GPU box): one rocprofv3 --pmc pass per
# counter (TCC_EA0_RDREQ total / 32B / 64B / 128B, the DRAM-bound subset, and
# WRITE_SIZE), so no pass can exceed the TCC block's counter slots.  Bytes read
# = 32 n32 + 64 n64 + 128 n128 -- a calibrated figure for access widths that
# FETCH_SIZE's fixed 64 B per request misreads (MI355X_MICROARCH.md "HBM":
# "other access widths are uncalibrated").
# usage: PASS_TIMEOUT=s tools/pmc_req.sh <outdir> <kernel-regex> <cmd...>
set -euo pipefail
OUT=$1; RX=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
for C in TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
         TCC_EA0_RDREQ_DRAM_sum WRITE_SIZE; do
  timeout -s KILL "${PASS_TIMEOUT:-300}" rocprofv3 --pmc $C --kernel-include-regex "$RX" --output-format csv \
      -d "$OUT/raw_$C" -o run -- "$@" > "$OUT/out_$C.log" 2>&1
  find "$OUT/raw_$C" -name "*counter_collection.csv" -exec cp {} "$OUT/counters_$C.csv" \;
  rm -rf "$OUT/raw_$C"
done
python3 tools/pmc_req_summarize.py "$OUT"
