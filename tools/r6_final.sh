#!/bin/bash
# Round-6 evidence on the final library (one GPU call per part; each step under its own
# limit, the first failure ends the part):
#   a: the GPU suite + smoke(), then tools/final_pmc.sh a (rocprof trace of the bench,
#      k_decode FETCH/WRITE, per-path LF traffic)
#   b: tools/final_pmc.sh b (request-size passes)
#   c: tools/r5_evidence_c.sh 1 (C2 / C5 traffic, the C3 bench line with the CPU baseline)
#   d: tools/r5_evidence_c.sh 2 (C2, C5, N = 1 sharded lines)
# usage: tools/r6_final.sh a|b|c|d
set -euo pipefail
O=gpurun_out/r06_final
mkdir -p "$O"
export TMPDIR=/tmp
case "$1" in
  a)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
    tail -2 "$O/gpu_tests.log"
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 \
        || { tail -30 "$O/smoke.log"; exit 1; }
    tail -1 "$O/smoke.log"
    bash tools/final_pmc.sh "$O" a ;;
  b) bash tools/final_pmc.sh "$O" b ;;
  c) bash tools/r5_evidence_c.sh "$O" 1 ;;
  d) bash tools/r5_evidence_c.sh "$O" 2 ;;
esac
echo "r6_final $1 done"
