set -o pipefail
# round 5, run v: the one-token AttnBlock fold test with the option held through the first forward
R=r05v
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "one_token" -x -v -s --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert|rel-L2" gpurun_out/$R/tests.log | head -20; exit 1; }
grep -E "passed|failed|folded" gpurun_out/$R/tests.log | tail -4
