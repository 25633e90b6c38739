set -o pipefail
# round 5, run d: p4<32> schedule variants (diagnostic build): B reads early, 9-slot A ring; and the lengthened C4 window test
R=r05d
mkdir -p gpurun_out/$R
timeout -k 10 400 python tools/census.py --n 256 --reps 1 --lib ab_libs/libitsd_hip_diag.so --variants "base,conv_dbg=823296,conv_dbg=831488,conv_dbg=839680" > gpurun_out/$R/ablate256.txt 2>&1 || { echo ablate_fail; tail -5 gpurun_out/$R/ablate256.txt; exit 1; }
grep variant gpurun_out/$R/ablate256.txt | tail -4
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_configs.py -k "C4" -x -v --timeout 250 --timeout-method thread > gpurun_out/$R/c4_tests.log 2>&1 || { echo tests_fail; tail -20 gpurun_out/$R/c4_tests.log; exit 1; }
tail -3 gpurun_out/$R/c4_tests.log
