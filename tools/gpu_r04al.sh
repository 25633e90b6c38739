set -o pipefail
R=r04al
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_attnblock.py tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread -k "attnblock or oracle" > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed|rel-L2|Error" gpurun_out/$R/tests.log | tail -22
