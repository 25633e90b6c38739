set -o pipefail
R=r04e
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u tools/fp32_archc_check.py --n 64 > gpurun_out/$R/fp32_check.txt 2>&1; echo "check rc=$?"; grep "n=" gpurun_out/$R/fp32_check.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rA > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed|FAIL|Error" gpurun_out/$R/tests.log | tail -12
timeout -k 10 200 python tools/census.py --n 64 --arch c > gpurun_out/$R/census_c64.txt 2>&1 || exit 1
grep -E "^total|launches" gpurun_out/$R/census_c64.txt | head -20
timeout -k 10 400 python tools/leg_time.py --legs C3 > gpurun_out/$R/legs.txt 2>&1 || exit 1
tail -2 gpurun_out/$R/legs.txt
