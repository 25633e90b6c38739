set -o pipefail
R=r04y
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -k "attention" > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/$R/tests.log
timeout -k 10 200 python tools/census.py --n 64 --arch c > gpurun_out/$R/c64.txt 2>&1 || exit 1
timeout -k 10 200 python tools/census.py --n 64 --arch c --set attn_wide=0 > gpurun_out/$R/c64_w0.txt 2>&1 || exit 1
grep -E "^total|attn" gpurun_out/$R/c64.txt gpurun_out/$R/c64_w0.txt
timeout -k 10 400 python tools/leg_time.py --legs C3 > gpurun_out/$R/c3.txt 2>&1 || exit 1
timeout -k 10 400 python tools/leg_time.py --legs C3 --set attn_wide=0 > gpurun_out/$R/c3_w0.txt 2>&1 || exit 1
tail -3 gpurun_out/$R/c3.txt gpurun_out/$R/c3_w0.txt
