#!/bin/bash
# Round-5 evidence on the final library, after tools/final_pmc.sh a / b (whose
# summaries are already under profiles/):
#   part 1: PMC traffic at C2 and C5, copied into profiles/ of this tree, then the
#           C3 bench line (the metric, with the CPU baseline, compact profile, C4 rehearsal);
#   part 2: the C2, C5 (PAQ-shaped) and N = 1 sharded bench lines (run after the C2 / C5
#           summaries of part 1 were copied into profiles/ of the sending tree).
# Each step under its own limit; the first failure ends it.
# usage: tools/r5_evidence_c.sh <outdir> 1|2
set -euo pipefail
O=$1
mkdir -p "$O"
if [ "$2" = 1 ]; then
  timeout -k 10 300 bash tools/pmc_traffic.sh "$O/pmc_c2" --tokens 3e8 --batch 32 > "$O/pmc_c2.log" 2>&1
  timeout -k 10 400 bash tools/pmc_traffic.sh "$O/pmc_c5" --corpus paq --tokens 1.5e9 --batch 2048 > "$O/pmc_c5.log" 2>&1
  cp "$O/pmc_c2/pmc_traffic.json" profiles/pmc_traffic_c2.json
  cp "$O/pmc_c5/pmc_traffic.json" profiles/pmc_traffic_c5.json
  echo "pmc c2 / c5 done"
  timeout -k 10 420 python3 bench.py > "$O/bench_c3.json" 2> "$O/bench_c3.log"
else
  timeout -k 10 240 python3 bench.py --tokens 3e8 --batch 32 --no-gather > "$O/bench_c2.json" 2> "$O/bench_c2.log"
  timeout -k 10 300 python3 bench.py --corpus paq --tokens 1.5e9 --batch 2048 --no-gather --no-rank21 \
      > "$O/bench_c5.json" 2> "$O/bench_c5.log"
  timeout -k 10 240 python3 bench.py --sharded-at-1 --tokens 1e9 --no-cpu --no-gather --no-rank21 \
      > "$O/bench_sharded1.json" 2> "$O/bench_sharded1.log"
fi
echo "r5_evidence_c $2 done"
