set -o pipefail
# round 5, run f: p5 k-step loads interleaved with its MFMAs (vs the compact-halo build); full-T parity with derived bounds
R=r05f
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests/test_gpu_p5.py tests/test_gpu_bench_configs.py -x -v --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; tail -30 gpurun_out/$R/tests.log; exit 1; }
tail -1 gpurun_out/$R/tests.log
for N in 32 64 256; do
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base > gpurun_out/$R/step${N}_new.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_compact.so > gpurun_out/$R/step${N}_compact.txt 2>&1 || { echo ab_old_fail; exit 1; }
done
timeout -k 10 200 python tools/step_ab.py --n 16 --img 64 --steps 20 --rounds 3 --variants base > gpurun_out/$R/stepC4_new.txt 2>&1 || { echo ab_fail; exit 1; }
timeout -k 10 200 python tools/step_ab.py --n 16 --img 64 --steps 20 --rounds 3 --variants base --lib ab_libs/libitsd_compact.so > gpurun_out/$R/stepC4_compact.txt 2>&1 || { echo ab_old_fail; exit 1; }
grep -H best gpurun_out/$R/step*.txt
timeout -k 10 200 python tools/census.py --n 32 --reps 3 > gpurun_out/$R/census32.txt 2>&1 || { echo census_fail; exit 1; }
timeout -k 10 200 python tools/census.py --n 32 --reps 3 --lib ab_libs/libitsd_r04.so > gpurun_out/$R/census32_r04.txt 2>&1 || { echo census_fail; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_T.py -k "not C5" -x -v -s --timeout 550 --timeout-method thread > gpurun_out/$R/fullT.log 2>&1 || { echo fullT_fail; grep -E "max\||rel-L2|FAIL" gpurun_out/$R/fullT.log | tail; exit 1; }
grep -E "C1|C2|passed|failed" gpurun_out/$R/fullT.log | tail -8
