# round 6: kernel trace of the world-1 sharded leg (B = 2048 only): per-kernel durations of the
# payload decode (with / without the fused signal) and the OR pass (with / without the flag wait)
set -o pipefail
export TMPDIR=/tmp
R=/tmp/r06_shprof
rm -rf $R
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R -o run -- python3 bench.py --sharded-at-1 --tokens 1e9 --no-cpu --no-gather --no-rank21 --no-c4 --sharded-batches 2048 > gpurun_out/r06_shprof.json 2> gpurun_out/r06_shprof.log || { tail -20 gpurun_out/r06_shprof.log; exit 1; }
find $R -name "*kernel_stats.csv" -exec cp {} gpurun_out/r06_shprof_stats.csv \;
T=$(find $R -name "*kernel_trace.csv" | head -1)
python3 - "$T" <<'PY'
import csv, sys, collections
seq = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if any(k in n for k in ("k_decode<true, true, 256", "k_or_rows")):
        g = r.get("Grid_Size", r.get("Grid_Size_X", ""))
        seq[(n[:60], g)].append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
for k, v in seq.items():
    v.sort()
    d = [x[1] for x in v]
    chunks = [sorted(d[i:i + 25]) for i in range(0, len(d), 25)]
    print(k, len(d), [round(c[len(c) // 2], 2) for c in chunks])
PY
PY
rm -rf $R
