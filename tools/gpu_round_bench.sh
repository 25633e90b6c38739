set -o pipefail
mkdir -p gpurun_out/r01 profiles
timeout -k 10 600 bash tools/pmc_passes.sh gpurun_out/r01/pmc --n 256 > gpurun_out/r01/pmc.log 2>&1 || { echo pmc_fail; exit 1; }
python tools/pmc_traffic.py gpurun_out/r01/pmc convgn profiles/pmc_traffic_convgn.json > gpurun_out/r01/traffic_convgn.json || exit 1
python tools/pmc_traffic.py gpurun_out/r01/pmc conv profiles/pmc_traffic_conv.json > gpurun_out/r01/traffic_conv.json || exit 1
python tools/pmc_traffic.py gpurun_out/r01/pmc convgnw profiles/pmc_traffic_convgnw.json > gpurun_out/r01/traffic_convgnw.json || exit 1
cp profiles/pmc_traffic_*.json gpurun_out/r01/
timeout -k 10 600 python bench.py > gpurun_out/r01/bench.json 2> gpurun_out/r01/bench.err || { echo bench_fail; tail -5 gpurun_out/r01/bench.err; exit 1; }
cat gpurun_out/r01/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01/prof -o bench -- python3 bench.py > gpurun_out/r01/prof_bench.json 2> gpurun_out/r01/prof.err || { echo prof_fail; tail -5 gpurun_out/r01/prof.err; exit 1; }
find gpurun_out/r01/prof -name "*kernel_trace.csv" -delete
ls -R gpurun_out/r01/prof | head
