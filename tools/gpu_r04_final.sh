set -o pipefail
R=${1:-r04f2}
mkdir -p gpurun_out/$R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$R/smoke.log 2>&1 || { echo smoke_fail; tail -5 gpurun_out/$R/smoke.log; exit 1; }
tail -1 gpurun_out/$R/smoke.log
bash tools/gpu_round_bench.sh $R
