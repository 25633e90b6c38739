set -o pipefail
# round 5, run m: 8x8 p4 on 96-cout tiles (256 tiles at N = 256) vs 128-cout (the previous build, m16all)
R=r05m
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "96_cout or full_batch or persistent" -x -v --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$R/tests.log | tail -2
for r in 1 2; do
  timeout -k 10 200 python tools/step_ab.py --n 256 --steps 30 --rounds 3 --variants base > gpurun_out/$R/step256_c96_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n 256 --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_m16all.so > gpurun_out/$R/step256_m16all_$r.txt 2>&1 || { echo ab_fail; exit 1; }
done
grep -H best gpurun_out/$R/step*.txt
timeout -k 10 200 python tools/census.py --n 256 --reps 3 > gpurun_out/$R/census256_c96.txt 2>&1 || { echo census_fail; exit 1; }
grep -E "p4_kernel<8" gpurun_out/$R/census256_c96.txt | head -12
