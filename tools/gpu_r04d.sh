set -o pipefail
R=r04d
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u tools/fp32_archc_check.py --n 2,64 --variants base,tap_prune=0,down_merge=0,tap_prune=0+down_merge=0 > gpurun_out/$R/fp32_check.txt 2>&1; echo "check rc=$?"; cat gpurun_out/$R/fp32_check.txt | grep "n="
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_configs.py -q --timeout 300 --timeout-method thread -rA > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "pruned|sub-pixel|passed|failed|FAIL|Error" gpurun_out/$R/tests.log | head -30
timeout -k 10 200 python tools/census.py --n 64 --arch c > gpurun_out/$R/census_c64.txt 2>&1 || exit 1
grep -E "^total|attn|conv H1|conv H2" gpurun_out/$R/census_c64.txt | head -20
timeout -k 10 400 python tools/leg_time.py --legs C3,C4 > gpurun_out/$R/legs.txt 2>&1 || exit 1
tail -4 gpurun_out/$R/legs.txt
