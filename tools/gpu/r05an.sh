set -o pipefail
# round 5, run an: conv3x3_gn_p5_kernel with an 18-slot A ring and 2 B buffers (r18 build) vs the shipped 9 / 3:
# parity on the variant (its own test run), census p5 times, step A/B at N = 256 / 32 / 64 and C4
R=r05an
mkdir -p gpurun_out/$R
ITSD_LIB=$PWD/ab_libs/libitsd_hip_r18.so timeout -k 10 400 python -u -m pytest tests/test_gpu_p5.py tests/test_gpu_p5_shortcut.py -x -q --timeout 250 --timeout-method thread > gpurun_out/$R/tests_r18.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests_r18.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$R/tests_r18.log | tail -1
for r in 1 2; do
for N in 256 32 64; do
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base > gpurun_out/$R/step${N}_main_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_r18.so > gpurun_out/$R/step${N}_r18_$r.txt 2>&1 || { echo ab_fail; exit 1; }
done
done
timeout -k 10 300 python tools/step_ab.py --n 16 --img 64 --steps 20 --rounds 3 --variants base > gpurun_out/$R/stepC4_main.txt 2>&1 || { echo ab_fail; exit 1; }
timeout -k 10 300 python tools/step_ab.py --n 16 --img 64 --steps 20 --rounds 3 --variants base --lib ab_libs/libitsd_hip_r18.so > gpurun_out/$R/stepC4_r18.txt 2>&1 || { echo ab_fail; exit 1; }
grep -H best gpurun_out/$R/step*.txt
for N in 256 32; do
for f in main r18; do
  LIB=""; [ $f = r18 ] && LIB="--lib ab_libs/libitsd_hip_r18.so"
  timeout -k 10 200 python tools/census.py --n $N --reps 3 $LIB > gpurun_out/$R/census${N}_$f.txt 2>&1 || { echo census_fail; exit 1; }
  grep -E "p5_kernel<" gpurun_out/$R/census${N}_$f.txt | awk -v f="$f $N" '{s[$NF]+=$9} END {for (k in s) printf "%s %s %.4f ms\n", f, k, s[k]}'
done
done
