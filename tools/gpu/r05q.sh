set -o pipefail
# round 5, run q: GroupNorm finalize loads batched (gn_coef / gn_apply) vs the previous build: C3 / C4 / N=32 steps,
# GroupNorm-path parity
R=r05q
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_configs.py -k "cfg or C3 or C4 or fp32 or gn" -x -q --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$R/tests.log | tail -2
for r in 1 2; do
  timeout -k 10 200 python tools/step_ab.py --arch c --n 32 --steps 20 --rounds 2 --variants base > gpurun_out/$R/stepC3_new_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --arch c --n 32 --steps 20 --rounds 2 --variants base --lib ab_libs/libitsd_hip_prev.so > gpurun_out/$R/stepC3_prev_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n 16 --img 64 --steps 20 --rounds 3 --variants base > gpurun_out/$R/stepC4_new_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n 16 --img 64 --steps 20 --rounds 3 --variants base --lib ab_libs/libitsd_hip_prev.so > gpurun_out/$R/stepC4_prev_$r.txt 2>&1 || { echo ab_fail; exit 1; }
done
grep -H best gpurun_out/$R/step*.txt
