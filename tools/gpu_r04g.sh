set -o pipefail
R=r04g
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -rA -k "attention_kernels or subpixel or full_configs or dead_tap" > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed|FAIL|Error" gpurun_out/$R/tests.log | head -20
timeout -k 10 200 python tools/census.py --n 16 --img 64 > gpurun_out/$R/census_c4.txt 2>&1 || exit 1
timeout -k 10 200 python tools/census.py --n 16 --img 64 --set attn_wide=0 > gpurun_out/$R/census_c4_nowide.txt 2>&1 || exit 1
grep -E "^total|attn" gpurun_out/$R/census_c4.txt gpurun_out/$R/census_c4_nowide.txt | head -30
timeout -k 10 200 python tools/census.py --n 64 --arch c > gpurun_out/$R/census_c64.txt 2>&1 || exit 1
timeout -k 10 200 python tools/census.py --n 64 --arch c --set attn_wide=2 > gpurun_out/$R/census_c64_wide2.txt 2>&1 || exit 1
grep -E "^total|attn" gpurun_out/$R/census_c64.txt gpurun_out/$R/census_c64_wide2.txt | head -40
timeout -k 10 400 python tools/leg_time.py --legs C3,C4 > gpurun_out/$R/legs.txt 2>&1 || exit 1
grep -E "^C[0-9]:" gpurun_out/$R/legs.txt
