set -o pipefail
R=r04f
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -rA -k "subpixel or dead_tap or convtranspose or full_configs or cfg" > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "split-K|pruned|passed|failed|FAIL|Error" gpurun_out/$R/tests.log | head -20
timeout -k 10 300 python tools/step_ab.py --n 32 --variants "base,subpix_split=0" --steps 100 > gpurun_out/$R/step32.txt 2>&1 || exit 1
tail -2 gpurun_out/$R/step32.txt
timeout -k 10 200 python tools/census.py --n 64 --arch c > gpurun_out/$R/census_c64.txt 2>&1 || exit 1
grep -E "^total|launches" gpurun_out/$R/census_c64.txt | head -20
timeout -k 10 200 python tools/census.py --n 16 --img 64 > gpurun_out/$R/census_c4.txt 2>&1 || exit 1
grep -E "^total|launches" gpurun_out/$R/census_c4.txt | head -20
timeout -k 10 400 python tools/leg_time.py --legs C3,C4 > gpurun_out/$R/legs.txt 2>&1 || exit 1
grep -E "^C[0-9]:" gpurun_out/$R/legs.txt
