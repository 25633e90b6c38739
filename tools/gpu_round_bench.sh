set -o pipefail
# Round-end measurement on one MI355X: GPU tests, PMC traffic passes, bench line, rocprof stats.
R=${1:-r01}
mkdir -p gpurun_out/$R profiles
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/$R/gpu_tests.log 2>&1 || { echo tests_fail; tail -20 gpurun_out/$R/gpu_tests.log; exit 1; }
tail -3 gpurun_out/$R/gpu_tests.log
timeout -k 10 600 bash tools/pmc_passes.sh gpurun_out/$R/pmc --n 256 > gpurun_out/$R/pmc.log 2>&1 || { echo pmc_fail; exit 1; }
for fam in convgnw convgnw4 convgn conv; do
  python tools/pmc_traffic.py gpurun_out/$R/pmc $fam profiles/pmc_traffic_$fam.json > gpurun_out/$R/traffic_$fam.json || echo "no $fam dispatches"
done
cp profiles/pmc_traffic_*.json gpurun_out/$R/
timeout -k 10 600 python bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { echo bench_fail; tail -5 gpurun_out/$R/bench.err; exit 1; }
cat gpurun_out/$R/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$R/prof -o bench -- python3 bench.py > gpurun_out/$R/prof_bench.json 2> gpurun_out/$R/prof.err || { echo prof_fail; tail -5 gpurun_out/$R/prof.err; exit 1; }
find gpurun_out/$R/prof -name "*kernel_trace.csv" -delete
ls -R gpurun_out/$R/prof | head
