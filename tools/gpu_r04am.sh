set -o pipefail
R=r04am
mkdir -p gpurun_out/$R
timeout -k 10 600 python tools/step_ab.py --n 16 --img 64 --variants "base,small_minks=2,small_minks=16,small_wide=0,small_wide=2,small_8x8=0,attn_wide=0,subpix_split=0,p4_w=15,attn_split=0" --steps 60 > gpurun_out/$R/step_c4.txt 2>&1 || exit 1
tail -n 10 gpurun_out/$R/step_c4.txt
timeout -k 10 600 python tools/step_ab.py --n 128 --variants "base,small_minks=2,small_wide=0,small_8x8=0,subpix_split=0,attn_split=0,conv1x1=0" --steps 40 > gpurun_out/$R/step128.txt 2>&1 || exit 1
tail -n 7 gpurun_out/$R/step128.txt
