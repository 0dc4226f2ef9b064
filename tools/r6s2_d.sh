#!/bin/bash
# round 6, session 2: the checked flag-barrier step (fm_peer_flags_step with sync) waiting by a
# spin on hipStreamQuery instead of hipStreamSynchronize -- world-1 sharded leg, A B A B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s2_d
mkdir -p $O
L=$PWD/fm-index-constrained-decoding_amd/fmidx
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_peer_exchange.py -m gpu \
    > $O/peer_tests.log 2>&1 || { tail -30 $O/peer_tests.log; exit 1; }
tail -1 $O/peer_tests.log
for v in _base "" _base ""; do
  FMIDX_LIB=$L/libfmidx$v.so timeout -k 10 300 python3 bench.py --sharded-at-1 --tokens 1e9 --no-cpu --no-gather --no-rank21 --no-c4 \
      > $O/sh$v.json 2> $O/sh$v.log || { tail -20 $O/sh$v.log; exit 1; }
  python3 - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r06s2_d/sh{sys.argv[1]}.json").read().strip().splitlines()[-1])
for b, x in d["sharded"]["by_global_batch"].items():
    print(sys.argv[1] or "spin", b, {m: round(y["ms_per_step"] * 1e3, 2) for m, y in x["modes"].items() if y.get("ms_per_step")}, x["masks_equal_unsharded"])
PY
done
