set -o pipefail
# round 5, run h: p4 on v_mfma_f32_16x16x32_bf16 (main lib: the 32x32 level) vs 32x32x16 (m32) vs all RES forms
# (m16all); calibration loops of both MFMA shapes; parity of the main lib
R=r05h
mkdir -p gpurun_out/$R
timeout -k 10 120 python -c "
from itsd import runtime as rt
for r in range(2):
    print('calib mfma 32x32x16 %.1f TF/s, 16x16x32 %.1f TF/s' % (rt.calibrate(rt.CALIB_MFMA_BF16), rt.calibrate(rt.CALIB_MFMA_BF16_16X16)))
" > gpurun_out/$R/calib.txt 2>&1 || { echo calib_fail; tail -5 gpurun_out/$R/calib.txt; exit 1; }
cat gpurun_out/$R/calib.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_configs.py -x -q --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests.log | head -20; exit 1; }
tail -1 gpurun_out/$R/tests.log
for N in 256 64; do
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base > gpurun_out/$R/step${N}_main.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_m32.so > gpurun_out/$R/step${N}_m32.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_m16all.so > gpurun_out/$R/step${N}_m16all.txt 2>&1 || { echo ab_fail; exit 1; }
done
grep -H best gpurun_out/$R/step*.txt
timeout -k 10 200 python tools/census.py --n 256 --reps 3 > gpurun_out/$R/census256_main.txt 2>&1 || { echo census_fail; exit 1; }
timeout -k 10 200 python tools/census.py --n 256 --reps 3 --lib ab_libs/libitsd_hip_m32.so > gpurun_out/$R/census256_m32.txt 2>&1 || { echo census_fail; exit 1; }
timeout -k 10 200 python tools/census.py --n 256 --reps 3 --lib ab_libs/libitsd_hip_m16all.so > gpurun_out/$R/census256_m16all.txt 2>&1 || { echo census_fail; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_T.py -k C5 -x -v -s --timeout 550 --timeout-method thread > gpurun_out/$R/c5.log 2>&1 || { echo c5_fail; grep -E "C5|assert" gpurun_out/$R/c5.log | tail; exit 1; }
grep -E "C5|passed|failed" gpurun_out/$R/c5.log | tail -8
