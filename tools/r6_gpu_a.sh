# round 6: the new GPU tests, then the A/Bs of the split emit (decode) and the persistent LF sweep (rank)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_r06.py tests/test_gpu_peer_exchange.py > gpurun_out/r06_t6.log 2>&1 || { tail -30 gpurun_out/r06_t6.log; exit 1; }
tail -3 gpurun_out/r06_t6.log
L=fm-index-constrained-decoding_amd/fmidx
timeout -k 10 600 python3 tools/ab_decode.py --reps 7 $L/libfmidx_nosplit.so $L/libfmidx.so $L/libfmidx_nosplit.so $L/libfmidx.so > gpurun_out/r06_ab_split.jsonl 2> gpurun_out/r06_ab_split.log || { tail -20 gpurun_out/r06_ab_split.log; exit 1; }
cut -c1-420 gpurun_out/r06_ab_split.jsonl
timeout -k 10 300 python3 tools/rank_queued.py --rank-only --works 2,4 --eager --reps 5 --out gpurun_out/r06_rank_persist.json > gpurun_out/r06_rank_persist.log 2>&1 || { tail -20 gpurun_out/r06_rank_persist.log; exit 1; }
FMIDX_LIB=$PWD/$L/libfmidx_pone.so timeout -k 10 300 python3 tools/rank_queued.py --rank-only --works 4 --eager --reps 5 --out gpurun_out/r06_rank_pone.json > gpurun_out/r06_rank_pone.log 2>&1 || { tail -20 gpurun_out/r06_rank_pone.log; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r06_rank_persist.json", "gpurun_out/r06_rank_pone.json"):
    d = json.load(open(f))
    for e in d["rank"]:
        print(f.split("/")[-1], e.get("lf_work"), e.get("pairs_log2"), "graph cold", round(e.get("cold_median_us", -1), 1),
              "eager cold", round(e.get("eager_cold_median_us", -1), 1), "eager warm", round(e.get("eager_warm_median_us", -1), 1),
              "exact", e.get("exact"), e.get("error", ""))
PY
