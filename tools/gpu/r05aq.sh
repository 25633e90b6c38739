set -o pipefail
# round 5, run aq: the shortcut-fold cost model's standalone-launch constant 5 chunk-times (sc5 build: also folds the
# 32x32 shortcuts at N = 32, the 8x8 ones at N = 64, the 4x4 ones at N = 256) vs the shipped 3; step A/B
R=r05aq
mkdir -p gpurun_out/$R
ITSD_LIB=$PWD/ab_libs/libitsd_hip_sc5.so timeout -k 10 400 python -u -m pytest tests/test_gpu_p5_shortcut.py -x -q --timeout 250 --timeout-method thread > gpurun_out/$R/tests_sc5.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests_sc5.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$R/tests_sc5.log | tail -1
for r in 1 2 3; do
for N in 32 64 256; do
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base > gpurun_out/$R/step${N}_main_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_sc5.so > gpurun_out/$R/step${N}_sc5_$r.txt 2>&1 || { echo ab_fail; exit 1; }
done
done
grep -H best gpurun_out/$R/step*.txt
