# round 6: the in-wave sweep at forced occupancy (6 / 8 waves per SIMD, spilling) against the default
set -o pipefail
export TMPDIR=/tmp
L=fm-index-constrained-decoding_amd/fmidx
for v in "" _wpe6 _wpe8; do
  FMIDX_LIB=$PWD/$L/libfmidx$v.so timeout -k 10 300 python3 tools/rank_queued.py --rank-only --works 2 --eager --reps 5 --out gpurun_out/r06_rank_wpe$v.json > gpurun_out/r06_rank_wpe$v.log 2>&1 || { tail -20 gpurun_out/r06_rank_wpe$v.log; exit 1; }
  python3 - "$v" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r06_rank_wpe{sys.argv[1]}.json"))
for e in d["rank"]:
    print(sys.argv[1] or "default", e.get("pairs_log2"), "eager cold", round(e.get("eager_cold_median_us", -1), 1), "exact", e.get("exact"))
PY
done
