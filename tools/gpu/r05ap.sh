set -o pipefail
# round 5, run ap (the final tree: + the tail coefficient layout): the whole GPU suite, PMC passes over one N=256 census forward,
# the bench line and rocprofv3 kernel stats of the same bench command
R=r05ap
mkdir -p gpurun_out/$R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.txt 2>&1 || { echo smoke_fail; tail -5 gpurun_out/$R/smoke.txt; exit 1; }
tail -2 gpurun_out/$R/smoke.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/$R/gpu_tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error" gpurun_out/$R/gpu_tests.log | tail -20; exit 1; }
tail -2 gpurun_out/$R/gpu_tests.log
timeout -k 10 600 bash tools/pmc_passes.sh gpurun_out/$R/pmc --n 256 > gpurun_out/$R/pmc.log 2>&1 || { echo pmc_fail; tail -5 gpurun_out/$R/pmc.log; exit 1; }
python tools/pmc_dispatch.py gpurun_out/$R/pmc > gpurun_out/$R/pmc_dispatch_table.txt || echo dispatch_table_fail
timeout -k 10 600 python bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { echo bench_fail; tail -5 gpurun_out/$R/bench.err; exit 1; }
tail -c 300 gpurun_out/$R/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$R/prof -o bench -- python3 bench.py --no-extras --no-cpu-baseline --no-live-traffic > gpurun_out/$R/prof_bench.json 2> gpurun_out/$R/prof.err || { echo prof_fail; tail -5 gpurun_out/$R/prof.err; exit 1; }
find gpurun_out/$R/prof -name "*kernel_trace.csv" -delete
find gpurun_out/$R/prof -name "*stats.csv"
