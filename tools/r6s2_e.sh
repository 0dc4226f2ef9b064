#!/bin/bash
# round 6, session 2: bench.py's peer preflight child, two processes on the one GPU, with the
# peer exchange's other cross-process tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s2_e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_peer_exchange.py -m gpu \
    > $O/peer_tests.log 2>&1 || { tail -40 $O/peer_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/peer_tests.log | tail -6
