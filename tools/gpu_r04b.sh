set -o pipefail
R=r04b
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u -m pytest tests/test_gpu_attnblock.py -q --timeout 200 --timeout-method thread -rA > gpurun_out/$R/attn_tests.log 2>&1; echo "attn tests rc=$?"; grep -E "split vs|forced|passed|failed" gpurun_out/$R/attn_tests.log
timeout -k 10 200 python tools/census.py --n 32 > gpurun_out/$R/census32_split.txt 2>&1 || exit 1
timeout -k 10 200 python tools/census.py --n 32 --set attn_split=0 > gpurun_out/$R/census32_nosplit.txt 2>&1 || exit 1
grep -E "attnblock|total" gpurun_out/$R/census32_split.txt gpurun_out/$R/census32_nosplit.txt
timeout -k 10 300 python tools/step_ab.py --n 32 --variants "base,attn_split=0" --steps 100 > gpurun_out/$R/step32.txt 2>&1 || exit 1
timeout -k 10 300 python tools/step_ab.py --n 64 --variants "base,attn_split=0" --steps 100 > gpurun_out/$R/step64.txt 2>&1 || exit 1
timeout -k 10 300 python tools/step_ab.py --n 256 --variants "base,p4_sub=0" --steps 30 > gpurun_out/$R/step256.txt 2>&1 || exit 1
tail -2 gpurun_out/$R/step32.txt gpurun_out/$R/step64.txt gpurun_out/$R/step256.txt
timeout -k 10 200 python tools/census.py --n 256 > gpurun_out/$R/census256.txt 2>&1 || exit 1
tail -16 gpurun_out/$R/census256.txt
