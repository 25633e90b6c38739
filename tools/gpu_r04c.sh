set -o pipefail
R=r04c
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_attnblock.py tests/test_gpu_parity.py tests/test_gpu_bench_configs.py -q --timeout 300 --timeout-method thread -rA > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "split vs|sub-pixel|passed|failed|FAIL" gpurun_out/$R/tests.log | head -20
timeout -k 10 300 python tools/step_ab.py --n 32 --variants "base,attn_split=0" --steps 100 > gpurun_out/$R/step32.txt 2>&1 || exit 1
tail -2 gpurun_out/$R/step32.txt
timeout -k 10 200 python tools/census.py --n 64 --arch c > gpurun_out/$R/census_c64.txt 2>&1 || exit 1
timeout -k 10 200 python tools/census.py --n 64 --arch c --set p4_sub=0 > gpurun_out/$R/census_c64_nosub.txt 2>&1 || exit 1
grep -E "^total" gpurun_out/$R/census_c64.txt gpurun_out/$R/census_c64_nosub.txt
timeout -k 10 200 python tools/census.py --n 256 --set p5=2 > gpurun_out/$R/census256_p5.txt 2>&1 || exit 1
timeout -k 10 200 python tools/census.py --n 256 --set conv_variant=3 > gpurun_out/$R/census256_cv3.txt 2>&1 || exit 1
timeout -k 10 200 python tools/census.py --n 256 > gpurun_out/$R/census256.txt 2>&1 || exit 1
grep -E "^total|H8 |conv H" gpurun_out/$R/census256*.txt
