set -o pipefail
R=r04a
mkdir -p gpurun_out/$R
timeout -k 10 720 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -rA > gpurun_out/$R/gpu_tests.log 2>&1
echo "tests rc=$?"
tail -3 gpurun_out/$R/gpu_tests.log
grep -E "full T|C2 bf16|bf16 pre-tail|window rel-L2" gpurun_out/$R/gpu_tests.log | head -20
timeout -k 10 420 python bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { echo bench_fail; tail -5 gpurun_out/$R/bench.err; exit 1; }
tail -c 400 gpurun_out/$R/bench.json
