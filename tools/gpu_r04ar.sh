set -o pipefail
R=r04ar
mkdir -p gpurun_out/$R
timeout -k 10 600 python bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { echo bench_fail; tail -5 gpurun_out/$R/bench.err; exit 1; }
tail -c 300 gpurun_out/$R/bench.json
