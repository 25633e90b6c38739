set -o pipefail
# Round measurement on one MI355X: GPU tests, PMC passes over one census forward (per-dispatch
# table + HBM traffic of the shipped kernels), the bench line, rocprofv3 kernel stats of the same
# bench command. Usage (GPU box): bash tools/gpu_round_bench.sh r02
R=${1:-r03}
mkdir -p gpurun_out/$R profiles
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/$R/gpu_tests.log 2>&1 || { echo tests_fail; tail -20 gpurun_out/$R/gpu_tests.log; exit 1; }
tail -3 gpurun_out/$R/gpu_tests.log
timeout -k 10 600 bash tools/pmc_passes.sh gpurun_out/$R/pmc --n 256 > gpurun_out/$R/pmc.log 2>&1 || { echo pmc_fail; tail -5 gpurun_out/$R/pmc.log; exit 1; }
python tools/pmc_dispatch.py gpurun_out/$R/pmc > gpurun_out/$R/pmc_dispatch_table.txt || echo dispatch_table_fail
for k in "conv3x3_gn_p4_kernel<32>" "conv3x3_gn_p4_kernel<16>" "conv3x3_gn_p4_kernel<8>" "conv_small<false>" \
         "conv_pipe<unsigned short, 2, true>" "conv1x1_stream_kernel<384, 4>" "conv1x1_stream_kernel<256, 4>" \
         "conv3x3_gn_p4_kernel<16, 128>" "attn_block_kernel<384>" "gn_apply_kernel" ; do
  f=$(echo "$k" | sed 's/[^A-Za-z0-9]/_/g; s/__*/_/g; s/_$//')
  python tools/pmc_traffic.py gpurun_out/$R/pmc "$k" gpurun_out/$R/pmc_traffic_$f.json > /dev/null || echo "no dispatches: $k"
done
timeout -k 10 600 python bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { echo bench_fail; tail -5 gpurun_out/$R/bench.err; exit 1; }
tail -c 600 gpurun_out/$R/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$R/prof -o bench -- python3 bench.py --no-extras --no-cpu-baseline --no-live-traffic > gpurun_out/$R/prof_bench.json 2> gpurun_out/$R/prof.err || { echo prof_fail; tail -5 gpurun_out/$R/prof.err; exit 1; }
find gpurun_out/$R/prof -name "*kernel_trace.csv" -delete
find gpurun_out/$R/prof -name "*stats.csv" | head
