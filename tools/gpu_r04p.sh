set -o pipefail
R=r04p
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_configs.py -q --timeout 300 --timeout-method thread -rA -k "p4_64x64 or 64 or A64 or archA64" > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "64x64|passed|failed|FAIL|Error" gpurun_out/$R/tests.log | head -12
timeout -k 10 200 python tools/census.py --n 16 --img 64 > gpurun_out/$R/census_c4.txt 2>&1 || exit 1
timeout -k 10 200 python tools/census.py --n 16 --img 64 --set p4_w=7 > gpurun_out/$R/census_c4_p5.txt 2>&1 || exit 1
grep -E "^total|H64" gpurun_out/$R/census_c4.txt gpurun_out/$R/census_c4_p5.txt | head -12
timeout -k 10 400 python tools/leg_time.py --legs C4 > gpurun_out/$R/legs.txt 2>&1 || exit 1
timeout -k 10 400 python tools/leg_time.py --legs C4 --set p4_w=7 > gpurun_out/$R/legs_p5.txt 2>&1 || exit 1
grep -E "^C[0-9]:" gpurun_out/$R/legs.txt gpurun_out/$R/legs_p5.txt
