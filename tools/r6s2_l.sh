#!/bin/bash
# round 6, session 2: the worklist LF form with the new tail kernel (k_lf_tail_sweep: 64 tail rows
# per wave, sweep_tails) -- LF parity variants, then lf_work -1 (in-wave) vs 1 (head sweep + tail
# kernel) at 2^19 / 2^21 pairs, then a kernel trace of lf_work 1 (head and tail apart)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s2_l
mkdir -p $O /tmp/prof_l
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "grouped_lf or workspace or sweep" \
    > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 400 python3 tools/rank_queued.py --rank-only --eager --works=-1,1,-1,1 --reps 5 --out $O/rank.json \
    > $O/rank.log 2>&1 || { tail -20 $O/rank.log; exit 1; }
grep pairs_log2 $O/rank.log | python3 -c "
import json, sys
for l in sys.stdin:
    e = json.loads(l); print(e['lf_work'], e['pairs_log2'], 'eager cold', round(e.get('eager_cold_median_us', 0), 1), 'eager warm', round(e.get('eager_warm_median_us', 0), 1), 'graph cold', round(e.get('cold_median_us', 0), 1), e.get('exact'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_l -o run -- python3 tools/rank_queued.py --rank-only --eager --works=1 --reps 5 \
    > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
t=$(find /tmp/prof_l -name "*kernel_trace.csv" | head -1)
python3 - "$t" <<'PY' | tee $O/lf_dispatches.txt | tail -12
import csv, sys
from collections import defaultdict
by = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    k = r.get("Kernel_Name", "")
    for name in ("k_lf_sweep", "k_lf_tail_sweep", "k_lf_tail"):
        if name + "<" in k or name + "(" in k:
            by[(name, r.get("Grid_Size", ""))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            break
for (name, g), d in sorted(by.items()):
    d2 = sorted(d)
    print(name, g, "n", len(d), "median", round(d2[len(d2) // 2], 1), "min", round(d2[0], 1), "max", round(d2[-1], 1))
PY
