set -o pipefail
# round 5, run o: p5 on v_mfma_f32_16x16x32_bf16 (main) vs 32x32x16 (p5m32 variant): p5 parity, step A/B
R=r05o
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests/test_gpu_p5.py tests/test_gpu_bench_configs.py -x -q --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$R/tests.log | tail -2
for N in 32 64 256; do
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base > gpurun_out/$R/step${N}_m16.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_p5m32.so > gpurun_out/$R/step${N}_m32.txt 2>&1 || { echo ab_fail; exit 1; }
done
timeout -k 10 200 python tools/step_ab.py --n 16 --img 64 --steps 20 --rounds 3 --variants base > gpurun_out/$R/stepC4_m16.txt 2>&1 || { echo ab_fail; exit 1; }
timeout -k 10 200 python tools/step_ab.py --n 16 --img 64 --steps 20 --rounds 3 --variants base --lib ab_libs/libitsd_hip_p5m32.so > gpurun_out/$R/stepC4_m32.txt 2>&1 || { echo ab_fail; exit 1; }
grep -H best gpurun_out/$R/step*.txt
