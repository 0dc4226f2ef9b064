# round 6: the persistent LF sweep A/B (own-queue drain), the 16-B transition slots (libfmidx_t16.so:
# parity suites + decode A/B + memory), the N = 1 sharded leg
set -o pipefail
export TMPDIR=/tmp
L=fm-index-constrained-decoding_amd/fmidx
FMIDX_LIB=$PWD/$L/libfmidx_t16.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_processors.py tests/test_gpu_r06.py tests/test_gpu_shard_processors.py -m gpu --deselect tests/test_gpu_parity.py::test_device_structs > gpurun_out/r06_t16_tests.log 2>&1 || { tail -30 gpurun_out/r06_t16_tests.log; exit 1; }
tail -2 gpurun_out/r06_t16_tests.log
timeout -k 10 600 python3 tools/ab_decode.py --reps 7 $L/libfmidx.so $L/libfmidx_t16.so $L/libfmidx.so $L/libfmidx_t16.so > gpurun_out/r06_ab_t16.jsonl 2> gpurun_out/r06_ab_t16.log || { tail -20 gpurun_out/r06_ab_t16.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r06_ab_t16.jsonl"):
    d = json.loads(l)
    print(d["lib"].split("/")[-1], "GiB", round(d["device_gib"], 2), "trans", round(d["trans_gib"], 2), d["trans_entries"], d["trans_dropped"],
          "cold", round(d["cold_median"], 2), "warm", round(d["warm_median"], 2), d["trace_ok"], d["mask_equal_first_lib"])
PY
timeout -k 10 300 python3 tools/rank_queued.py --rank-only --works 2,4 --eager --reps 5 --out gpurun_out/r06_rank_persist2.json > gpurun_out/r06_rank_persist2.log 2>&1 || { tail -20 gpurun_out/r06_rank_persist2.log; exit 1; }
FMIDX_LIB=$PWD/$L/libfmidx_t16.so timeout -k 10 300 python3 tools/rank_queued.py --rank-only --works 2 --eager --reps 5 --out gpurun_out/r06_rank_t16.json > gpurun_out/r06_rank_t16.log 2>&1 || { tail -20 gpurun_out/r06_rank_t16.log; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r06_rank_persist2.json", "gpurun_out/r06_rank_t16.json"):
    d = json.load(open(f))
    for e in d["rank"]:
        print(f.split("/")[-1], e.get("lf_work"), e.get("pairs_log2"), "eager cold", round(e.get("eager_cold_median_us", -1), 1),
              "eager warm", round(e.get("eager_warm_median_us", -1), 1), "exact", e.get("exact"), e.get("error", ""))
PY
