#!/bin/bash
# kernel-trace A/B of the class-list LF launch across library variants:
# tools/ab_lists.sh lib1.so lib2.so ... -> gpurun_out/ab_lists/<lib>.txt (+ .json)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_lists
for lib in "$@"; do
  name=$(basename "$lib" .so)
  rm -rf /tmp/rw_prof
  FMIDX_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/rw_prof -o rw -- \
    python3 -u tools/lf_lists_probe.py > gpurun_out/ab_lists/$name.json 2> gpurun_out/ab_lists/$name.err
  python3 tools/trace_summ.py gpurun_out/ab_lists/$name.txt
  grep -c k_lf gpurun_out/ab_lists/$name.txt
done
