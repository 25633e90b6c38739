set -o pipefail
R=r04i
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -rA -k "streaming_1x1 or small_wide or bf16_full_batch" > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed|FAIL|Error" gpurun_out/$R/tests.log | head -20
timeout -k 10 300 python tools/step_ab.py --n 256 --variants "base,conv1x1=0" --steps 30 > gpurun_out/$R/step256.txt 2>&1 || exit 1
tail -2 gpurun_out/$R/step256.txt
timeout -k 10 200 python tools/census.py --n 256 > gpurun_out/$R/census256.txt 2>&1 || exit 1
grep -E "^total|launches|conv1x1" gpurun_out/$R/census256.txt
