#!/bin/bash
# The round's whole evidence set on the final library, in one GPU call: the hash-stamped PMC
# passes (tools/final_pmc.sh a and b, C2 / C5 traffic), their summaries copied into profiles/ of
# this tree (so the bench lines that follow read them), the bench lines (tools/r4_measure.sh),
# the GPU test suite and smoke().  Each step under its own limit; the first failure ends it.
# usage: tools/r4_evidence.sh <outdir>
set -euo pipefail
O=$1
mkdir -p "$O"
bash tools/final_pmc.sh "$O" a
bash tools/final_pmc.sh "$O" b
timeout -k 10 500 bash tools/pmc_traffic.sh "$O/pmc_c2" --tokens 3e8 --batch 32 > "$O/pmc_c2.log" 2>&1
timeout -k 10 600 bash tools/pmc_traffic.sh "$O/pmc_c5" --corpus paq --tokens 1.5e9 --batch 2048 > "$O/pmc_c5.log" 2>&1
cp "$O/pmc_c3/pmc_traffic.json" profiles/pmc_traffic.json
cp "$O/pmc_c2/pmc_traffic.json" profiles/pmc_traffic_c2.json
cp "$O/pmc_c5/pmc_traffic.json" profiles/pmc_traffic_c5.json
cp "$O/pmc_rank/pmc_rank.json" profiles/pmc_rank.json
cp "$O/req_c3/pmc_req.json" profiles/pmc_req_c3.json
cp "$O/req_rank/pmc_req.json" profiles/pmc_req_rank.json
echo "pmc done"
bash tools/r4_measure.sh "$O/bench"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
echo "r4_evidence done"
