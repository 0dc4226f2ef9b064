set -euo pipefail
O=gpurun_out/c2s; mkdir -p $O
run() { n=$1; shift; env "$@" timeout -k 10 200 python3 bench.py --tokens 3e8 --batch 32 --no-gather --no-cpu --no-c4 --no-rank21 > $O/$n.json 2> $O/$n.log; }
run base FMIDX_X=0
run t512s16 FMIDX_DEC_THREADS=512 FMIDX_MASK_SLICES=16
run t256s32 FMIDX_DEC_THREADS=256 FMIDX_MASK_SLICES=32
run t1024s4 FMIDX_DEC_THREADS=1024 FMIDX_MASK_SLICES=4
run t512s8 FMIDX_DEC_THREADS=512 FMIDX_MASK_SLICES=8
run t1024s16 FMIDX_DEC_THREADS=1024 FMIDX_MASK_SLICES=16
run base2 FMIDX_X=0
