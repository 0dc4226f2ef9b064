# round 6: footprint knobs on the 16-B slot build (C3): cache_min 8192 / 16384, trans_min 2
set -o pipefail
export TMPDIR=/tmp
L=fm-index-constrained-decoding_amd/fmidx/libfmidx.so
timeout -k 10 900 python3 tools/ab_decode.py --reps 7 $L "$L@cache_min=8192" "$L@cache_min=16384" "$L@transitions=2,trans_min=2" $L \
    > gpurun_out/r06_ab_fp.jsonl 2> gpurun_out/r06_ab_fp.log || { tail -20 gpurun_out/r06_ab_fp.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r06_ab_fp.jsonl"):
    d = json.loads(l)
    print(d["lib"].split("/")[-1], d.get("build_options"), "GiB", round(d["device_gib"], 2), "trans", round(d["trans_gib"], 2), d["trans_entries"], d["trans_dropped"],
          "cold", round(d["cold_median"], 2), "warm", round(d["warm_median"], 2), d["trace_ok"], d["mask_equal_first_lib"])
PY
