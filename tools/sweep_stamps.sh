set -e
for T in 64 128 256 512; do
 for SW in 8032 16032 32768; do
  QUIET=1 STAMPS_LIB=libfmidx_stamps_t$T.so FMIDX_MASK_SW=$SW timeout -k 10 120 python tools/probe_stamps.py 2>&1 | grep SUMMARY
 done
done
