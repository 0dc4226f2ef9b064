#!/bin/bash
# One GPU-box pass (gpurun): the -m gpu tests, smoke(), the default bench and
# (optionally) its rocprofv3 kernel-trace summary, each under its own time
# limit.  A test FAILURE (pytest rc 1) still lets the later steps run; a
# crash, abort, fault or time-out (any other non-zero rc) ends the pass.
# usage: tools/gpu_check.sh <tag> [tests|smoke|bench|prof]...   (default: all four)
set -uo pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
STEPS=("$@")
[ ${#STEPS[@]} -eq 0 ] && STEPS=(tests smoke bench prof)
export TMPDIR=/tmp
for s in "${STEPS[@]}"; do
  echo "[gpu_check] $s $(date +%T)"
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
             > "$OUT/pytest.log" 2>&1; rc=$?
           tail -3 "$OUT/pytest.log"
           [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    smoke) timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
           tail -2 "$OUT/smoke.log" ;;
    bench) timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log" || exit $?
           cat "$OUT/bench.log" | grep -v amdgpu.ids ;;
    prof)  timeout -k 10 600 tools/profile_bench.sh "$OUT/prof" --no-gather || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "[gpu_check] done $(date +%T)"
