#!/bin/bash
# The round's hash-stamped counter evidence (run after the last kernel change;
# every file is stamped with the libfmidx.so hash and bench.py uses it only for
# that build), in two GPU calls:
#   part a: rocprof kernel trace of the bench, FETCH/WRITE traffic of k_decode,
#           per-path FETCH/WRITE of the grouped LF launch
#   part b: request-size passes of the bench (k_decode and its rank-at-scale
#           grouped LF launch) and of tools/probe_rank.py's per-path launches
# usage: tools/final_pmc.sh <outdir> a|b
set -euo pipefail
O=$1
mkdir -p "$O"
export TMPDIR=/tmp
if [ "$2" = a ]; then
  timeout -k 10 300 bash tools/profile_bench.sh "$O/prof" > "$O/prof.log" 2>&1
  timeout -k 10 400 bash tools/pmc_traffic.sh "$O/pmc_c3" > "$O/pmc_c3.log" 2>&1
  timeout -k 10 200 bash tools/pmc_rank.sh "$O/pmc_rank" > "$O/pmc_rank.log" 2>&1
else
  PASS_TIMEOUT=120 timeout -k 10 700 bash tools/pmc_req.sh "$O/req_c3" "k_decode|k_lf_group|k_lf_sweep" \
      python3 bench.py --no-cpu --no-c4 --no-gather --eager-replay > "$O/req_c3.log" 2>&1
  PASS_TIMEOUT=90 timeout -k 10 450 bash tools/pmc_req.sh "$O/req_rank" "k_lf_group|k_lf_sweep" \
      python3 tools/probe_rank.py --rows-log2 19 --patterns 1024 --by-path --out "$O/req_rank/probe.json" \
      > "$O/req_rank.log" 2>&1
fi
echo "final_pmc $2 done"
