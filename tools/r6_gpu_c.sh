# round 6: persistent LF sweep v3 (fetch-and-add claims, 64 queues): parity, then the rank A/B
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_r06.py -m gpu -k persist \
    > gpurun_out/r06_p3_tests.log 2>&1 || { tail -30 gpurun_out/r06_p3_tests.log; exit 1; }
tail -1 gpurun_out/r06_p3_tests.log
timeout -k 10 300 python3 tools/rank_queued.py --rank-only --works 2,4 --eager --reps 5 --out gpurun_out/r06_rank_persist3.json \
    > gpurun_out/r06_rank_persist3.log 2>&1 || { tail -20 gpurun_out/r06_rank_persist3.log; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r06_rank_persist3.json"))
for e in d["rank"]:
    print(e.get("lf_work"), e.get("pairs_log2"), "eager cold", round(e.get("eager_cold_median_us", -1), 1),
          "eager warm", round(e.get("eager_warm_median_us", -1), 1), "exact", e.get("exact"), e.get("error", ""))
PY
