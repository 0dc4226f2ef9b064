# round 6: the OR pass's flag wait without the system-scope acquire fence (buffer_inv sc0 sc1 in every
# workgroup; all peer reads are system-scope loads): peer-exchange tests on that build, then the
# world-1 sharded leg A/B
set -o pipefail
export TMPDIR=/tmp
L=fm-index-constrained-decoding_amd/fmidx
FMIDX_LIB=$PWD/$L/libfmidx_noacq.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_or.py tests/test_gpu_peer_exchange.py tests/test_gpu_shard_processors.py -m gpu \
    > gpurun_out/r06_noacq_tests.log 2>&1 || { tail -30 gpurun_out/r06_noacq_tests.log; exit 1; }
tail -1 gpurun_out/r06_noacq_tests.log
for v in "" _noacq "" _noacq; do
  FMIDX_LIB=$PWD/$L/libfmidx$v.so timeout -k 10 300 python3 bench.py --sharded-at-1 --tokens 1e9 --no-cpu --no-gather --no-rank21 --no-c4 > gpurun_out/r06_acq$v.json 2> gpurun_out/r06_acq$v.log || { tail -20 gpurun_out/r06_acq$v.log; exit 1; }
  python3 - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r06_acq{sys.argv[1]}.json").read().strip().splitlines()[-1])
for b, x in d["sharded"]["by_global_batch"].items():
    print(sys.argv[1] or "fence", b, {m: round(y["ms_per_step"] * 1e3, 2) for m, y in x["modes"].items() if y.get("ms_per_step")}, x["masks_equal_unsharded"])
PY
done
