#!/bin/bash
# round 6, session 2: cold phase stamps of the decode step with the absent-symbol probe shortcut
# off (FMIDX_PROBE_COMPLETE=0) and on (the default)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s2_b
mkdir -p $O
for pc in 0 1; do
  FMIDX_PROBE_COMPLETE=$pc COLD=1 timeout -k 10 300 python3 tools/probe_stamps.py > $O/stamps_pc$pc.log 2>&1 || { tail -20 $O/stamps_pc$pc.log; exit 1; }
  grep "kernel span" $O/stamps_pc$pc.log | sed "s/^/[pc$pc] /"
done
