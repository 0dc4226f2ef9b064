#!/bin/bash
# Round-4 bench lines on the final library (GPU box): C3 (the metric, with the CPU
# baseline), C2, C5 (PAQ-shaped), and the sharded path at N = 1.  Each step under
# its own time limit; the first failure ends the script.
# usage: tools/r4_measure.sh <outdir>
set -euo pipefail
O=$1
mkdir -p "$O"
timeout -k 10 420 python3 bench.py > "$O/bench_c3.json" 2> "$O/bench_c3.log"
timeout -k 10 240 python3 bench.py --tokens 3e8 --batch 32 --no-gather > "$O/bench_c2.json" 2> "$O/bench_c2.log"
timeout -k 10 300 python3 bench.py --corpus paq --tokens 1.5e9 --batch 2048 --no-gather --no-rank21 \
    > "$O/bench_c5.json" 2> "$O/bench_c5.log"
timeout -k 10 240 python3 bench.py --sharded-at-1 --tokens 1e9 --no-cpu --no-gather --no-rank21 \
    > "$O/bench_sharded1.json" 2> "$O/bench_sharded1.log"
echo "r4_measure done"
