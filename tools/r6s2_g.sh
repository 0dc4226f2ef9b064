#!/bin/bash
# round 6, session 2: the in-wave LF sweep as a grid-stride loop over resident waves
# (FMIDX_SWEEP_GRID workgroups; 0 = one per 256-row block, the default kernel), 2^19 / 2^21 pairs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s2_g
mkdir -p $O
for g in 0 1024 512 0 1024 2048; do
  FMIDX_SWEEP_GRID=$g timeout -k 10 300 python3 tools/rank_queued.py --rank-only --eager --works=-1 --reps 5 \
      --out $O/grid$g.json > $O/grid$g.log 2>&1 || { tail -20 $O/grid$g.log; exit 1; }
  grep pairs_log2 $O/grid$g.log | python3 -c "
import json, sys
for l in sys.stdin:
    e = json.loads(l); print('grid $g', e['pairs_log2'], 'graph cold', round(e.get('cold_median_us', 0), 1), 'eager cold', round(e.get('eager_cold_median_us', 0), 1), 'eager warm', round(e.get('eager_warm_median_us', 0), 1), e.get('exact'))"
done
