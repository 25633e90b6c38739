set -o pipefail
R=r04w
mkdir -p gpurun_out/$R
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_search.py tests/test_gpu_bench_configs.py -q --timeout 300 --timeout-method thread -k "attention or cfg or archC or full_configs or trajectory or window or search or dead_tap" > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/$R/tests.log
timeout -k 10 300 python tools/step_ab.py --n 256 --variants "base,tail_px=64" --steps 30 > gpurun_out/$R/step256.txt 2>&1 || exit 1
tail -2 gpurun_out/$R/step256.txt
timeout -k 10 300 python tools/step_ab.py --n 32 --variants "base,tail_px=64" --steps 100 > gpurun_out/$R/step32.txt 2>&1 || exit 1
tail -2 gpurun_out/$R/step32.txt
timeout -k 10 200 python tools/census.py --n 64 --arch c > gpurun_out/$R/c64.txt 2>&1 || exit 1
grep -E "^total|attn_flash|attn_cs" gpurun_out/$R/c64.txt
timeout -k 10 200 python tools/census.py --n 16 --img 64 > gpurun_out/$R/c4.txt 2>&1 || exit 1
grep -E "^total|attn_cs" gpurun_out/$R/c4.txt
