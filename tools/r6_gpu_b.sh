# round 6: the persistent LF sweep A/B (own-queue drain) and the N = 1 sharded leg
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_r06.py -k persist > gpurun_out/r06_t7.log 2>&1 || { tail -30 gpurun_out/r06_t7.log; exit 1; }
tail -2 gpurun_out/r06_t7.log
timeout -k 10 300 python3 tools/rank_queued.py --rank-only --works 2,4 --eager --reps 5 --out gpurun_out/r06_rank_persist2.json > gpurun_out/r06_rank_persist2.log 2>&1 || { tail -20 gpurun_out/r06_rank_persist2.log; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r06_rank_persist2.json"))
for e in d["rank"]:
    print(e.get("lf_work"), e.get("pairs_log2"), "eager cold", round(e.get("eager_cold_median_us", -1), 1),
          "eager warm", round(e.get("eager_warm_median_us", -1), 1), "exact", e.get("exact"), e.get("error", ""))
PY
timeout -k 10 240 python3 bench.py --sharded-at-1 --tokens 1e9 --no-cpu --no-gather --no-rank21 --no-c4 > gpurun_out/r06_sharded1d.json 2> gpurun_out/r06_sharded1d.log || { tail -20 gpurun_out/r06_sharded1d.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06_sharded1d.json").read().strip().splitlines()[-1])
for B, r in d["sharded"]["by_global_batch"].items():
    print("B", B, "best", r["exchange"], round(r["ms_per_step"] * 1e3, 1))
    for m, x in r["modes"].items():
        print("   ", m, round(x["ms_per_step"] * 1e3, 1) if x.get("ms_per_step") else x.get("error"), x.get("masks_equal_unsharded"))
PY
