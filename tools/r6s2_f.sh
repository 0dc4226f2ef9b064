#!/bin/bash
# round 6, session 2: the LF launch at 2^19 / 2^21 pairs, in-wave sweep (lf_work -1) against the
# sweep + worklist tail (lf_work 1, direct launches), then a rocprof kernel trace of the latter
# (the head-only sweep and the tail kernel timed apart)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s2_f
mkdir -p $O
timeout -k 10 400 python3 tools/rank_queued.py --rank-only --eager --works=-1,1 --reps 5 --out $O/rank_w1.json \
    > $O/rank_w1.log 2>&1 || { tail -20 $O/rank_w1.log; exit 1; }
grep pairs_log2 $O/rank_w1.log | python3 -c "
import json, sys
for l in sys.stdin:
    e = json.loads(l); print(e['lf_work'], e['pairs_log2'], 'graph cold', round(e.get('cold_median_us', 0), 1), 'eager cold', round(e.get('eager_cold_median_us', 0), 1), 'eager warm', round(e.get('eager_warm_median_us', 0), 1), e.get('exact'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/rank_queued.py --rank-only --eager --works=1 --reps 5 \
    > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
grep -E "k_lf_sweep|k_lf_tail" $O/kernel_stats.csv | cut -c1-200
