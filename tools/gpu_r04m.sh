set -o pipefail
R=r04m
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_attnblock.py -q --timeout 300 --timeout-method thread -rA -k "small_8x8 or small_wide or split_attnblock or subpixel" > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "8x8|passed|failed|FAIL|Error" gpurun_out/$R/tests.log | head -12
timeout -k 10 300 python tools/step_ab.py --n 32 --variants "base,small_8x8=0" --steps 100 > gpurun_out/$R/step32.txt 2>&1 || exit 1
tail -2 gpurun_out/$R/step32.txt
timeout -k 10 300 python tools/step_ab.py --n 64 --variants "base,small_8x8=0" --steps 100 > gpurun_out/$R/step64.txt 2>&1 || exit 1
tail -2 gpurun_out/$R/step64.txt
timeout -k 10 300 python tools/step_ab.py --n 128 --variants "base,small_8x8=0" --steps 50 > gpurun_out/$R/step128.txt 2>&1 || exit 1
tail -2 gpurun_out/$R/step128.txt
timeout -k 10 200 python tools/census.py --n 32 > gpurun_out/$R/census32.txt 2>&1 || exit 1
grep -E "^total|launches" gpurun_out/$R/census32.txt
