set -o pipefail
# round 5, run ao: tail_mfma_kernel's GroupNorm coefficients staged [4][C/8][4] (main) vs [C/8][16] (cfl0 build):
# smoke, parity, PMC conflicts, census tail time, step A/B N = 256 and C3
R=r05ao
mkdir -p gpurun_out/$R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.txt 2>&1 || { echo smoke_fail; tail -5 gpurun_out/$R/smoke.txt; exit 1; }
tail -1 gpurun_out/$R/smoke.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_search.py tests/test_gpu_bench_configs.py -x -q --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$R/tests.log | tail -1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in main cfl0; do
  LIB=""; [ $L = cfl0 ] && LIB="--lib ab_libs/libitsd_hip_cfl0.so"
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES --output-format csv -d gpurun_out/$R/pmc_$L -o run -- python3 tools/census.py --reps 1 --n 256 $LIB > gpurun_out/$R/pmc_$L.log 2>&1 || { echo pmc_fail $L; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for L in ("main", "cfl0"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); names = {}
    for fn in glob.glob(f"gpurun_out/r05ao/pmc_{L}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "tail" in r["Kernel_Name"]:
                acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"]); names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0]
    for d, c in acc.items(): print(L, names[d], {k: "%.3g" % v for k, v in c.items()})
PY
for r in 1 2; do
  timeout -k 10 200 python tools/step_ab.py --n 256 --steps 30 --rounds 3 --variants base > gpurun_out/$R/step256_main_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n 256 --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_cfl0.so > gpurun_out/$R/step256_cfl0_$r.txt 2>&1 || { echo ab_fail; exit 1; }
done
timeout -k 10 200 python tools/step_ab.py --arch c --n 32 --steps 20 --rounds 3 --variants base > gpurun_out/$R/stepC3_main.txt 2>&1 || { echo ab_fail; exit 1; }
timeout -k 10 200 python tools/step_ab.py --arch c --n 32 --steps 20 --rounds 3 --variants base --lib ab_libs/libitsd_hip_cfl0.so > gpurun_out/$R/stepC3_cfl0.txt 2>&1 || { echo ab_fail; exit 1; }
grep -H best gpurun_out/$R/step*.txt
for f in main cfl0; do
  LIB=""; [ $f = cfl0 ] && LIB="--lib ab_libs/libitsd_hip_cfl0.so"
  timeout -k 10 200 python tools/census.py --n 256 --reps 3 $LIB > gpurun_out/$R/census256_$f.txt 2>&1 || { echo census_fail; exit 1; }
  grep -E " tail " gpurun_out/$R/census256_$f.txt | head -1 | sed "s/^/$f /"
done
