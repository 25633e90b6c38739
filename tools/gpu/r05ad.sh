set -o pipefail
# round 5, run ad: 8x8 p4 (16x16x32 compact forms) padding lanes on 8 zero rows by residue (main) vs one zero row
# (zr0 build): parity, SQ_LDS_BANK_CONFLICT, step A/B at N = 256 / 128; p5 forced K-slice counts at N = 32 / 64
R=r05ad
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_configs.py -k "persistent or full_batch or 96_cout or interior or headline or compact" -x -q --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$R/tests.log | tail -2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in main zr0; do
  LIB=""; [ $L = zr0 ] && LIB="--lib ab_libs/libitsd_hip_zr0.so"
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES --output-format csv -d gpurun_out/$R/pmc_$L -o run -- python3 tools/census.py --reps 1 --n 256 $LIB > gpurun_out/$R/pmc_$L.log 2>&1 || { echo pmc_fail $L; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for L in ("main", "zr0"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); names = {}
    for fn in glob.glob(f"gpurun_out/r05ad/pmc_{L}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "conv3x3_gn_p4_kernel" in r["Kernel_Name"]:
                acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"]); names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for d, c in acc.items():
        for k, v in c.items(): per[names[d]][k].append(v)
    for n, c in sorted(per.items()):
        print(L, n, len(c["SQ_LDS_BANK_CONFLICT"]), {k: "%.3g" % (sum(v) / len(v)) for k, v in c.items()})
PY
for r in 1 2; do
for N in 256 128; do
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base > gpurun_out/$R/step${N}_main_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_zr0.so > gpurun_out/$R/step${N}_zr0_$r.txt 2>&1 || { echo ab_fail; exit 1; }
done
done
grep -H best gpurun_out/$R/step*.txt
for N in 32 64; do
  timeout -k 10 300 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants "base,p5_split=2,p5_split=4,p5_split=8" > gpurun_out/$R/p5split${N}.txt 2>&1 || { echo ab_fail; exit 1; }
done
grep -H best gpurun_out/$R/p5split*.txt
