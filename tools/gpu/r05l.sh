set -o pipefail
# round 5, run l: attn_block_kernel phase timeline at N = 256 (stamps build)
R=r05l
mkdir -p gpurun_out/$R
timeout -k 10 200 python tools/attn_timeline.py ab_libs/libitsd_hip_stamps.so --n 256 > gpurun_out/$R/attn_timeline256.txt 2>&1 || { echo tl_fail; tail -5 gpurun_out/$R/attn_timeline256.txt; exit 1; }
cat gpurun_out/$R/attn_timeline256.txt
