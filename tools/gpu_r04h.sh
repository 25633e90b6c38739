set -o pipefail
R=r04h
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_attnblock.py -q --timeout 300 --timeout-method thread -rA -k "small_wide or attention or split_attnblock" > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "wide|passed|failed|FAIL|Error" gpurun_out/$R/tests.log | head -20
timeout -k 10 300 python tools/step_ab.py --n 32 --variants "base,small_wide=0" --steps 100 > gpurun_out/$R/step32.txt 2>&1 || exit 1
tail -2 gpurun_out/$R/step32.txt
timeout -k 10 300 python tools/step_ab.py --n 64 --variants "base,small_wide=0" --steps 100 > gpurun_out/$R/step64.txt 2>&1 || exit 1
tail -2 gpurun_out/$R/step64.txt
timeout -k 10 300 python tools/step_ab.py --n 256 --variants "base,small_wide=0" --steps 30 > gpurun_out/$R/step256.txt 2>&1 || exit 1
tail -2 gpurun_out/$R/step256.txt
timeout -k 10 200 python tools/census.py --n 32 > gpurun_out/$R/census32.txt 2>&1 || exit 1
grep -E "^total|launches" gpurun_out/$R/census32.txt
timeout -k 10 200 python tools/census.py --n 64 --arch c --set attn_wide_nq=1 > gpurun_out/$R/census_c64_nq1.txt 2>&1 || exit 1
timeout -k 10 200 python tools/census.py --n 64 --arch c > gpurun_out/$R/census_c64.txt 2>&1 || exit 1
grep -E "^total|attn_cs" gpurun_out/$R/census_c64.txt gpurun_out/$R/census_c64_nq1.txt
timeout -k 10 200 python tools/census.py --n 16 --img 64 --set attn_wide_nq=2 > gpurun_out/$R/census_c4_nq2.txt 2>&1 || exit 1
grep -E "^total|attn_cs" gpurun_out/$R/census_c4_nq2.txt
