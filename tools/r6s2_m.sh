#!/bin/bash
# round 6, session 2: the worklist LF form with k_lf_tail_sweep at kTailRows = 4 / 8 / 16 rows per
# wave (libfmidx.so / _r8 / _r16): parity variants on the R = 4 library, then lf_work -1 vs 1
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s2_m
mkdir -p $O
L=$PWD/fm-index-constrained-decoding_amd/fmidx
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "grouped_lf or workspace or sweep" \
    > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in "" _r8 _r16; do
  FMIDX_LIB=$L/libfmidx$v.so timeout -k 10 400 python3 tools/rank_queued.py --rank-only --eager --works=-1,1,-1,1 --reps 5 --out $O/rank$v.json \
      > $O/rank$v.log 2>&1 || { tail -20 $O/rank$v.log; exit 1; }
  grep pairs_log2 $O/rank$v.log | python3 -c "
import json, sys
for l in sys.stdin:
    e = json.loads(l); print('lib$v', e['lf_work'], e['pairs_log2'], 'eager cold', round(e.get('eager_cold_median_us', 0), 1), 'eager warm', round(e.get('eager_warm_median_us', 0), 1), e.get('exact'))"
done
