set -o pipefail
# round 5, run x: the bf16 MFMA tail at 512 threads (8 waves, one 16-pixel group each) vs 256 (tail256 variant)
R=r05x
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_search.py -k "trajectory or search or cfg or full_batch" -x -q --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$R/tests.log | tail -2
for r in 1 2; do
  timeout -k 10 200 python tools/step_ab.py --n 256 --steps 30 --rounds 3 --variants base > gpurun_out/$R/step256_t512_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n 256 --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_tail256.so > gpurun_out/$R/step256_t256_$r.txt 2>&1 || { echo ab_fail; exit 1; }
done
grep -H best gpurun_out/$R/step*.txt
timeout -k 10 200 python tools/census.py --n 256 --reps 3 > gpurun_out/$R/census256_t512.txt 2>&1 || { echo census_fail; exit 1; }
timeout -k 10 200 python tools/census.py --n 256 --reps 3 --lib ab_libs/libitsd_hip_tail256.so > gpurun_out/$R/census256_t256.txt 2>&1 || { echo census_fail; exit 1; }
grep -H "tail " gpurun_out/$R/census256_*.txt | head -4
