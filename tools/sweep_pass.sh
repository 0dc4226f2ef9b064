set -euo pipefail
O=gpurun_out/sp; mkdir -p $O
L=fm-index-constrained-decoding_amd/fmidx
for v in sp1 sp3 sp4; do
FMIDX_TUNING=lf_work=2 FMIDX_LIB=$L/libfmidx_$v.so timeout -k 10 300 python3 tools/probe_rank.py --rows-log2 19,21 --patterns 4096 --out $O/$v.json > $O/$v.log 2>&1
done
FMIDX_TUNING=lf_work=2 timeout -k 10 300 python3 tools/probe_rank.py --rows-log2 19,21 --patterns 4096 --out $O/sp2.json > $O/sp2.log 2>&1
