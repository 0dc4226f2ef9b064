#!/bin/bash
# One GPU-box pass (gpurun): the -m gpu tests, smoke(), the default bench and
# (optionally) its rocprofv3 kernel-trace summary, each under its own time
# limit.  A test FAILURE (pytest rc 1) still lets the later steps run; a
# crash, abort, fault or time-out (any other non-zero rc) ends the pass.
# usage: tools/gpu_check.sh <tag> [tests|smoke|bench|prof|c2|c5|pmc|pmc_c2|service|proc]...
#        (default: tests smoke bench prof)
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
    c2)    timeout -k 10 300 python -u bench.py --tokens 3e8 --batch 32 --no-gather > "$OUT/c2.json" 2> "$OUT/c2.log" || exit $?
           grep "step cold" "$OUT/c2.log" ;;
    c5)    timeout -k 10 300 python -u bench.py --tokens 1.5e9 --batch 2048 --no-gather > "$OUT/c5.json" 2> "$OUT/c5.log" || exit $?
           grep "step cold" "$OUT/c5.log" ;;
    pmc)   timeout -k 10 600 tools/pmc_traffic.sh "$OUT/pmc_c3" --no-gather || exit $?
           cat "$OUT/pmc_c3/pmc_traffic.json" ;;
    pmc_c2) timeout -k 10 600 tools/pmc_traffic.sh "$OUT/pmc_c2" --tokens 3e8 --batch 32 --no-gather || exit $? ;;
    service) timeout -k 10 300 python -u tools/bench_service.py > "$OUT/service.json" 2> "$OUT/service.log" || exit $?
           cat "$OUT/service.json" ;;
    proc)  timeout -k 10 300 python -u tools/bench_processor.py > "$OUT/proc.json" 2> "$OUT/proc.log" || exit $?
           cat "$OUT/proc.json" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "[gpu_check] done $(date +%T)"
