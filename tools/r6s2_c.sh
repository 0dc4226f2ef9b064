#!/bin/bash
# round 6, session 2: the GPU suite on the library with the absent-symbol probe shortcut and its
# completeness flag export (tests/test_gpu_r06.py::test_probe_complete_absent_vs_oracle)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s2_c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_r06.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > $O/r06.log 2>&1 || { tail -40 $O/r06.log; exit 1; }
tail -3 $O/r06.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
