# round 6: the static split of the wide rows' emit at 512-thread workgroups (two per CU, so a row's
# helper is co-resident instead of dispatched after the rows retire), against the default geometry
# and the 512-thread two-slice geometry; split parity first
set -o pipefail
export TMPDIR=/tmp
L=fm-index-constrained-decoding_amd/fmidx
FMIDX_LIB=$PWD/$L/libfmidx_split.so FMIDX_TUNING=dec_threads=512,mask_slices=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_r06.py -m gpu -k split \
    > gpurun_out/r06_s512_tests.log 2>&1 || { tail -30 gpurun_out/r06_s512_tests.log; exit 1; }
tail -1 gpurun_out/r06_s512_tests.log
timeout -k 10 700 python3 tools/ab_decode.py --reps 7 $L/libfmidx.so "$L/libfmidx.so%dec_threads=512" "$L/libfmidx_split.so%dec_threads=512,mask_slices=1" \
    $L/libfmidx.so "$L/libfmidx.so%dec_threads=512" "$L/libfmidx_split.so%dec_threads=512,mask_slices=1" \
    > gpurun_out/r06_ab_s512.jsonl 2> gpurun_out/r06_ab_s512.log || { tail -20 gpurun_out/r06_ab_s512.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r06_ab_s512.jsonl"):
    d = json.loads(l)
    print(d["lib"].split("/")[-1], d.get("tuning"), "cold", round(d["cold_median"], 2), "warm", round(d["warm_median"], 2), d["trace_ok"], d["mask_equal_first_lib"])
PY
