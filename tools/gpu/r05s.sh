set -o pipefail
# round 5, run s: the 8x8 p4 launches' XCD-grouped tile order (p4_xcd = 2: a pixel tile's 4 cout tiles on one XCD)
# vs the default: step A/B in one process, and each setting's HBM traffic (FETCH_SIZE x 2 + WRITE_SIZE) per launch
R=r05s
mkdir -p gpurun_out/$R
timeout -k 10 300 python tools/step_ab.py --n 256 --steps 30 --rounds 4 --variants "base,p4_xcd=2" > gpurun_out/$R/step256_xcd.txt 2>&1 || { echo ab_fail; exit 1; }
grep best gpurun_out/$R/step256_xcd.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 2; do
  for P in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/$R/pmc_xcd$v/$P -o run -- python3 tools/census.py --reps 1 --n 256 --set p4_xcd=$v > gpurun_out/$R/pmc_xcd${v}_$P.log 2>&1 || { echo pmc_fail; tail -3 gpurun_out/$R/pmc_xcd${v}_$P.log; exit 1; }
  done
  python tools/pmc_traffic.py gpurun_out/$R/pmc_xcd$v "conv3x3_gn_p4_kernel<8, 512>" gpurun_out/$R/traffic8_xcd$v.json > /dev/null && cat gpurun_out/$R/traffic8_xcd$v.json
done
find gpurun_out/$R -name "*.csv" -size +2M -delete
