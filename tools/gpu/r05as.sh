set -o pipefail
# round 5, run as: the whole GPU suite on the shipped tree (after the fold constant 5)
R=r05as
mkdir -p gpurun_out/$R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/$R/gpu_tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error" gpurun_out/$R/gpu_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/$R/gpu_tests.log
