set -o pipefail
# round 5, run z: p4 stage hand-offs by per-wave LDS counters (main) vs the block barrier (noflags variant)
R=r05z
mkdir -p gpurun_out/$R
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_configs.py -k "persistent or full_batch or 96_cout or subpixel or headline or sweep or C3 or C5" -x -q --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$R/tests.log | tail -2
for r in 1 2; do
for N in 256 128; do
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base > gpurun_out/$R/step${N}_flags_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_noflags.so > gpurun_out/$R/step${N}_barrier_$r.txt 2>&1 || { echo ab_fail; exit 1; }
done
done
grep -H best gpurun_out/$R/step*.txt
timeout -k 10 200 python tools/census.py --n 256 --reps 3 > gpurun_out/$R/census256_flags.txt 2>&1 || { echo census_fail; exit 1; }
timeout -k 10 200 python tools/census.py --n 256 --reps 3 --lib ab_libs/libitsd_hip_noflags.so > gpurun_out/$R/census256_barrier.txt 2>&1 || { echo census_fail; exit 1; }
for f in flags barrier; do grep -E "p4_kernel<" gpurun_out/$R/census256_$f.txt | awk -v f=$f '{s[$NF]+=$9} END {for (k in s) printf "%s %s %.4f ms\n", f, k, s[k]}'; done
