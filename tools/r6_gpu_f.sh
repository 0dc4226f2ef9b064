# round 6: the flag-barrier step as one C call (fm_peer_flags_step): the peer-exchange and sharded
# processor GPU tests, then the world-1 sharded leg
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_peer_exchange.py tests/test_gpu_shard_processors.py tests/test_gpu_r06.py -m gpu \
    > gpurun_out/r06_fused_tests.log 2>&1 || { tail -30 gpurun_out/r06_fused_tests.log; exit 1; }
tail -1 gpurun_out/r06_fused_tests.log
timeout -k 10 300 python3 bench.py --sharded-at-1 --tokens 1e9 --no-cpu --no-gather --no-rank21 > gpurun_out/r06_sharded_fused.json 2> gpurun_out/r06_sharded_fused.log || { tail -20 gpurun_out/r06_sharded_fused.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06_sharded_fused.json").read().strip().splitlines()[-1])
for b, v in d["sharded"]["by_global_batch"].items():
    print(b, {m: round(x["ms_per_step"] * 1e3, 2) for m, x in v["modes"].items() if x.get("ms_per_step")}, v["masks_equal_unsharded"])
print("replica", d["ms_per_step"] * 1e3)
PY
