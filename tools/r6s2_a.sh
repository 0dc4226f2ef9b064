#!/bin/bash
# round 6, session 2: the absent-symbol probe shortcut (kProbeComplete: a probe miss beside a
# free slot ends the step).  GPU suite on the new library, then the C3 decode A/B against the
# session's base library (masks compared step by step), then bench rank legs of both.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s2_a
mkdir -p $O
L=$PWD/fm-index-constrained-decoding_amd/fmidx
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u tools/ab_decode.py --reps 7 $L/libfmidx_base.so $L/libfmidx.so $L/libfmidx_base.so $L/libfmidx.so \
    > $O/ab.json 2> $O/ab.log || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.json
for v in _base "" _base ""; do
  FMIDX_LIB=$L/libfmidx$v.so timeout -k 10 400 python3 bench.py --no-cpu --no-gather --no-c4 > $O/bench$v.json 2> $O/bench$v.log || { tail -20 $O/bench$v.log; exit 1; }
  grep -E "step cold|rank" $O/bench$v.log | sed "s/^/[$v] /"
done
