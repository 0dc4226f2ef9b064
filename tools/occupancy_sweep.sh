#!/bin/bash
# Rank (LF) launches at forced occupancy: the in-wave sweep and
# the grouped kernel built with amdgpu_waves_per_eu (make qvariant NAME=sw6
# VFLAGS=-DFMIDX_SWEEP_WPE=6, ...), each timed by tools/probe_rank.py at 2^17,
# 2^19, 2^21 pairs on the C3 index.  usage: tools/occupancy_sweep.sh <outdir>
set -euo pipefail
O=$1
mkdir -p "$O"
L=fm-index-constrained-decoding_amd/fmidx
R="--rows-log2 17,19,21 --patterns 4096"
FMIDX_TUNING=lf_work=2 timeout -k 10 300 python3 tools/probe_rank.py $R --by-path --out "$O/sweep_base.json" > "$O/sweep_base.log" 2>&1
FMIDX_TUNING=lf_work=2 FMIDX_LIB=$L/libfmidx_sw6.so timeout -k 10 300 python3 tools/probe_rank.py $R --out "$O/sweep_w6.json" > "$O/sweep_w6.log" 2>&1
FMIDX_TUNING=lf_work=2 FMIDX_LIB=$L/libfmidx_sw8.so timeout -k 10 300 python3 tools/probe_rank.py $R --out "$O/sweep_w8.json" > "$O/sweep_w8.log" 2>&1
FMIDX_TUNING=lf_work=0 timeout -k 10 300 python3 tools/probe_rank.py $R --by-path --out "$O/group_base.json" > "$O/group_base.log" 2>&1
FMIDX_TUNING=lf_work=0 FMIDX_LIB=$L/libfmidx_gr5.so timeout -k 10 300 python3 tools/probe_rank.py $R --out "$O/group_w5.json" > "$O/group_w5.log" 2>&1
FMIDX_TUNING=lf_work=0 FMIDX_LIB=$L/libfmidx_gr6.so timeout -k 10 300 python3 tools/probe_rank.py $R --out "$O/group_w6.json" > "$O/group_w6.log" 2>&1
echo occupancy_sweep done
