#!/bin/bash
# round 6, session 2: kernel trace of the worklist LF form (lf_work 1: the head-only sweep, then the
# tail kernel), direct launches at 2^19 / 2^21 pairs -- the two kernels' durations apart
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s2_k
mkdir -p $O /tmp/prof_k
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_k -o run -- python3 tools/rank_queued.py --rank-only --eager --works=1 --reps 5 \
    > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find /tmp/prof_k -name "*kernel_stats.csv" | head -1)
cp "$f" $O/kernel_stats.csv
t=$(find /tmp/prof_k -name "*kernel_trace.csv" | head -1)
python3 - "$t" <<'PY' > $O/lf_dispatches.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    k = r.get("Kernel_Name", "")
    if "k_lf_sweep" in k or "k_lf_tail" in k:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print(k.split("(")[0][-40:], r.get("Grid_Size", r.get("Grid_Size_X", "")), round(d, 1))
PY
cat $O/lf_dispatches.txt | tail -40
