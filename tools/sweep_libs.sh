#!/bin/bash
# A/B timing of decode-kernel variants on the GPU box: each argument is
# LIBNAME[:ENV=VAL[,ENV=VAL...]]; one bench --no-cpu run each, step line only.
# usage: tools/sweep_libs.sh libfmidx_base.so libfmidx.so:FMIDX_EARLY_ZERO_WIDTH=512
set -euo pipefail
PKG=fm-index-constrained-decoding_amd/fmidx
for spec in "$@"; do
  lib=${spec%%:*}
  envs=""
  [[ "$spec" == *:* ]] && envs=${spec#*:}
  echo "== $spec"
  env FMIDX_LIB=$PWD/$PKG/$lib ${envs//,/ } timeout -k 10 240 python3 bench.py --no-cpu ${BENCH_ARGS:-} 2>&1 >/dev/null | grep "step "
done
