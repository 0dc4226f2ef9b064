#!/bin/bash
# (round 5: FMIDX_OR_PERPART is a compile-time variant now -- make ... VFLAGS=-DFMIDX_OR_PERPART=0 and FMIDX_LIB)
# The OR pass's sparse lists per part (FMIDX_OR_PERPART=1) vs over one flat index space (0):
# GPU tests of the exchange, the synthetic OR micro-bench and the C4 rehearsal, both ways.
set -euo pipefail
O=$1
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_or.py \
    tests/test_gpu_peer_exchange.py tests/test_gpu_shard_processors.py > "$O/tests.log" 2>&1
for v in 1 0; do
  FMIDX_OR_PERPART=$v timeout -k 10 120 python3 tools/bench_or_rows.py > "$O/or_syn_$v.json" 2>&1
  FMIDX_OR_PERPART=$v timeout -k 10 120 python3 tools/bench_or_rows.py --wide 0.15 --mean 400 > "$O/or_wide_$v.json" 2>&1
  FMIDX_OR_PERPART=$v timeout -k 10 480 python3 bench.py --no-cpu --no-gather --no-rank21 > "$O/c3c4_$v.json" 2> "$O/c3c4_$v.log"
done
echo "or_perpart_ab done"
