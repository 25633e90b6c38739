set -o pipefail
# round 5, run b: the GPU suite after the pruning + fail-loud hand-off + p5 A-fragment buffer loads; step A/Bs vs the round-4 build
R=r05b
mkdir -p gpurun_out/$R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$R/gpu_tests.log 2>&1 || { echo tests_fail; tail -30 gpurun_out/$R/gpu_tests.log; exit 1; }
tail -3 gpurun_out/$R/gpu_tests.log
for N in 256 32 64; do
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base > gpurun_out/$R/step${N}_new.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_r04.so > gpurun_out/$R/step${N}_r04.txt 2>&1 || { echo ab_old_fail; exit 1; }
done
grep -h best gpurun_out/$R/step*.txt
