set -e
# (round 5: FMIDX_EARLY_ZERO_WIDTH is a compile-time variant now -- make variant NAME=ez VFLAGS=-DFMIDX_EARLY_ZERO_WIDTH=512)
for EW in 0 64 1000000000000; do
  echo "EARLY_ZERO_WIDTH=$EW"
  FMIDX_EARLY_ZERO_WIDTH=$EW timeout -k 10 200 python bench.py --no-cpu 2>&1 >/dev/null | grep step
  FMIDX_EARLY_ZERO_WIDTH=$EW QUIET=1 timeout -k 10 200 python tools/probe_stamps.py 2>&1 | grep SUMMARY
done
