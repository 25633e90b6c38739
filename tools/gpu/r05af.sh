set -o pipefail
# round 5, run af: conv3x3_gn_p5_kernel launch timelines (stamps build) at N = 256 (the 4x4 level: 15 % of the forward)
# and N = 32 (every level), after the shortcut fold
R=r05af
mkdir -p gpurun_out/$R
timeout -k 10 300 python tools/timeline.py ab_libs/libitsd_hip_stamps.so --n 256 > gpurun_out/$R/p5_timeline_n256.txt 2>&1 || { echo tl_fail; tail -5 gpurun_out/$R/p5_timeline_n256.txt; exit 1; }
timeout -k 10 300 python tools/timeline.py ab_libs/libitsd_hip_stamps.so --n 32 > gpurun_out/$R/p5_timeline_n32.txt 2>&1 || { echo tl_fail; tail -5 gpurun_out/$R/p5_timeline_n32.txt; exit 1; }
head -40 gpurun_out/$R/p5_timeline_n256.txt
# the shipped tree against the tree before the shortcut fold (prefold: commit 69bdb2d), same box: p5<4> at N = 256 runs no fold
for r in 1 2; do
  timeout -k 10 200 python tools/step_ab.py --n 256 --steps 30 --rounds 3 --variants base > gpurun_out/$R/step256_main_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n 256 --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_prefold.so > gpurun_out/$R/step256_prefold_$r.txt 2>&1 || { echo ab_fail; exit 1; }
done
grep -H best gpurun_out/$R/step*.txt
timeout -k 10 200 python tools/census.py --n 256 --reps 3 > gpurun_out/$R/census256_main.txt 2>&1 || { echo census_fail; exit 1; }
timeout -k 10 200 python tools/census.py --n 256 --reps 3 --lib ab_libs/libitsd_hip_prefold.so > gpurun_out/$R/census256_prefold.txt 2>&1 || { echo census_fail; exit 1; }
for f in main prefold; do grep -E "p5_kernel<|p4_kernel<" gpurun_out/$R/census256_$f.txt | awk -v f=$f '{s[$NF]+=$9} END {for (k in s) printf "%s %s %.4f ms\n", f, k, s[k]}'; done
