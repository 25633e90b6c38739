set -o pipefail
# round 5, run am: conv3x3_gn_p5_kernel launch timelines (stamps build) after the per-level halo swizzle, N = 256 / 32
R=r05am
mkdir -p gpurun_out/$R
timeout -k 10 300 python tools/timeline.py ab_libs/libitsd_hip_stamps.so --n 256 > gpurun_out/$R/p5_timeline_n256.txt 2>&1 || { echo tl_fail; tail -5 gpurun_out/$R/p5_timeline_n256.txt; exit 1; }
timeout -k 10 300 python tools/timeline.py ab_libs/libitsd_hip_stamps.so --n 32 > gpurun_out/$R/p5_timeline_n32.txt 2>&1 || { echo tl_fail; tail -5 gpurun_out/$R/p5_timeline_n32.txt; exit 1; }
sed -n 20,40p gpurun_out/$R/p5_timeline_n256.txt
