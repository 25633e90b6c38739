set -o pipefail
R=r04x
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -k "tail_64px" > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/$R/tests.log
timeout -k 10 400 python tools/step_ab.py --n 256 --variants "base,tail_px=64,conv1x1=0,p4_sub=0" --steps 30 > gpurun_out/$R/step256.txt 2>&1 || exit 1
tail -4 gpurun_out/$R/step256.txt
timeout -k 10 500 python tools/step_ab.py --n 32 --variants "base,tail_px=64,small_wide=0,subpix_split=0,small_8x8=0,attn_split=0" --steps 100 > gpurun_out/$R/step32.txt 2>&1 || exit 1
tail -6 gpurun_out/$R/step32.txt
timeout -k 10 500 python tools/step_ab.py --n 64 --variants "base,small_wide=0,subpix_split=0,small_8x8=0,attn_split=0" --steps 100 > gpurun_out/$R/step64.txt 2>&1 || exit 1
tail -5 gpurun_out/$R/step64.txt
timeout -k 10 200 python tools/census.py --n 64 --arch c > gpurun_out/$R/c64.txt 2>&1 || exit 1
grep -E "^total|attn_flash|attn_cs" gpurun_out/$R/c64.txt
