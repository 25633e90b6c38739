set -o pipefail
# round 5, run p: (1) parity of the p5 16x16x32 form, the attention prefetch and the 96-cout 8x8 tiles; (2) attention
# launches, new vs the previous build (m16all); (3) p5 16x16x32 (main) vs 32x32x16 (p5m32) step A/Bs
R=r05p
mkdir -p gpurun_out/$R
timeout -k 10 500 python -u -m pytest tests/test_gpu_p5.py tests/test_gpu_bench_configs.py tests/test_gpu_attnblock.py tests/test_gpu_parity.py -k "p5 or C3 or C4 or C5 or attn or 96_cout or full_batch" -x -q --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$R/tests.log | tail -2
timeout -k 10 200 python tools/census.py --n 256 --reps 3 > gpurun_out/$R/census256_new.txt 2>&1 || { echo census_fail; exit 1; }
timeout -k 10 200 python tools/census.py --n 256 --reps 3 --lib ab_libs/libitsd_hip_m16all.so > gpurun_out/$R/census256_old.txt 2>&1 || { echo census_fail; exit 1; }
grep -H "attnblock  launches\|convgn H4" gpurun_out/$R/census256_*.txt
for N in 32 64 256; do
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base > gpurun_out/$R/step${N}_m16.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_p5m32.so > gpurun_out/$R/step${N}_m32.txt 2>&1 || { echo ab_fail; exit 1; }
done
timeout -k 10 200 python tools/step_ab.py --n 16 --img 64 --steps 20 --rounds 3 --variants base > gpurun_out/$R/stepC4_m16.txt 2>&1 || { echo ab_fail; exit 1; }
timeout -k 10 200 python tools/step_ab.py --n 16 --img 64 --steps 20 --rounds 3 --variants base --lib ab_libs/libitsd_hip_p5m32.so > gpurun_out/$R/stepC4_m32.txt 2>&1 || { echo ab_fail; exit 1; }
grep -H best gpurun_out/$R/step*.txt
