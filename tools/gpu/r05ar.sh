set -o pipefail
# round 5, run ar: the shipped tree after the fold constant 5: smoke, the p5 / shortcut / attention / bench-config tests
R=r05ar
mkdir -p gpurun_out/$R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.txt 2>&1 || { echo smoke_fail; tail -5 gpurun_out/$R/smoke.txt; exit 1; }
tail -1 gpurun_out/$R/smoke.txt
timeout -k 10 700 python -u -m pytest tests/test_gpu_p5_shortcut.py tests/test_gpu_p5.py tests/test_gpu_attnblock.py tests/test_gpu_bench_configs.py tests/test_gpu_search.py -x -q --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$R/tests.log | tail -1
timeout -k 10 300 python tools/step_ab.py --n 32 --steps 30 --rounds 3 --variants "base,p5_sc=0" > gpurun_out/$R/step32.txt 2>&1 || { echo ab_fail; exit 1; }
grep best gpurun_out/$R/step32.txt
