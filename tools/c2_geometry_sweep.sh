set -euo pipefail
O=gpurun_out/c2s; mkdir -p $O
run() { n=$1; shift; env "$@" timeout -k 10 200 python3 bench.py --tokens 3e8 --batch 32 --no-gather --no-cpu --no-c4 --no-rank21 > $O/$n.json 2> $O/$n.log; }
run base FMIDX_X=0
run t512s16 FMIDX_TUNING=dec_threads=512,mask_slices=16
run t256s32 FMIDX_TUNING=dec_threads=256,mask_slices=32
run t1024s4 FMIDX_TUNING=dec_threads=1024,mask_slices=4
run t512s8 FMIDX_TUNING=dec_threads=512,mask_slices=8
run t1024s16 FMIDX_TUNING=dec_threads=1024,mask_slices=16
run base2 FMIDX_X=0
