set -o pipefail
# round 5, run e: compact interior halo (8x8 / 16x16 p4) + the 8x8 level on the LDS residual / drain path
R=r05e
mkdir -p gpurun_out/$R
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_configs.py tests/test_gpu_p5.py -x -v --timeout 300 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|error" gpurun_out/$R/tests.log | head -20; tail -30 gpurun_out/$R/tests.log; exit 1; }
tail -2 gpurun_out/$R/tests.log
for N in 256 1024; do
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 20 --rounds 3 --variants base > gpurun_out/$R/step${N}_new.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 20 --rounds 3 --variants base --lib ab_libs/libitsd_abuf.so > gpurun_out/$R/step${N}_abuf.txt 2>&1 || { echo ab_old_fail; exit 1; }
done
grep -h best gpurun_out/$R/step*.txt
timeout -k 10 200 python tools/census.py --n 256 --reps 3 > gpurun_out/$R/census256.txt 2>&1 || { echo census_fail; exit 1; }
timeout -k 10 200 python tools/census.py --n 256 --reps 3 --lib ab_libs/libitsd_abuf.so > gpurun_out/$R/census256_abuf.txt 2>&1 || { echo census_fail; exit 1; }
grep -A20 "^total" gpurun_out/$R/census256.txt | head -12; grep -A20 "^total" gpurun_out/$R/census256_abuf.txt | head -12
