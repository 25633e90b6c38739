set -o pipefail
R=r04k
mkdir -p gpurun_out/$R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rA > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed|FAIL|Error" gpurun_out/$R/tests.log | tail -8
timeout -k 10 300 python tools/step_ab.py --n 256 --variants "base,conv1x1=2,conv1x1=0" --steps 30 > gpurun_out/$R/step256.txt 2>&1 || exit 1
tail -3 gpurun_out/$R/step256.txt
timeout -k 10 200 python tools/census.py --n 256 > gpurun_out/$R/census256.txt 2>&1 || exit 1
timeout -k 10 200 python tools/census.py --n 256 --set conv1x1=2 > gpurun_out/$R/census256_ns7.txt 2>&1 || exit 1
grep -E "^total|conv1x1|tail|head" gpurun_out/$R/census256.txt gpurun_out/$R/census256_ns7.txt
timeout -k 10 300 python tools/step_ab.py --n 32 --variants "base" --steps 100 > gpurun_out/$R/step32.txt 2>&1 || exit 1
tail -1 gpurun_out/$R/step32.txt
