set -o pipefail
R=r04l
mkdir -p gpurun_out/$R
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_full_T.py tests/test_gpu_bench_configs.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -rA > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed|FAIL|Error" gpurun_out/$R/tests.log | tail -6
timeout -k 10 200 python tools/census.py --n 256 > gpurun_out/$R/census256.txt 2>&1 || exit 1
grep -E "^total|tail|head" gpurun_out/$R/census256.txt
timeout -k 10 200 python tools/census.py --n 64 --arch c --set gn_wide=2 > gpurun_out/$R/census_c64_gnwide2.txt 2>&1 || exit 1
timeout -k 10 200 python tools/census.py --n 64 --arch c > gpurun_out/$R/census_c64.txt 2>&1 || exit 1
grep -E "^total" gpurun_out/$R/census_c64_gnwide2.txt gpurun_out/$R/census_c64.txt
timeout -k 10 300 python tools/step_ab.py --n 256 --variants "base" --steps 30 > gpurun_out/$R/step256.txt 2>&1 || exit 1
tail -1 gpurun_out/$R/step256.txt
