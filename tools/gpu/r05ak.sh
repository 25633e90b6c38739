set -o pipefail
# round 5, run ak (= aj + ai): p4's non-compact 8x8 / 16x16 halo (sub-pixel forms) swizzled by halo coordinates (main) vs
# (h >> 1) & 7 (subswz0 build): parity (sub-pixel / ConvTranspose2d tests, C3), PMC, census, step A/B N = 256 and C3
R=r05aj
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_configs.py -k "subpix or convt or transpose or upsample or headline or C3 or archC" -x -q --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$R/tests.log | tail -2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in main subswz0; do
  LIB=""; [ $L = subswz0 ] && LIB="--lib ab_libs/libitsd_hip_subswz0.so"
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES --output-format csv -d gpurun_out/$R/pmc_$L -o run -- python3 tools/census.py --reps 1 --n 256 $LIB > gpurun_out/$R/pmc_$L.log 2>&1 || { echo pmc_fail $L; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for L in ("main", "subswz0"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); names = {}
    for fn in glob.glob(f"gpurun_out/r05aj/pmc_{L}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "conv3x3_gn_p4_kernel" in r["Kernel_Name"] and ("128>" in r["Kernel_Name"] or "384>" in r["Kernel_Name"]):
                acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"]); names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0]
    for d, c in acc.items(): print(L, names[d], {k: "%.3g" % v for k, v in c.items()})
PY
for r in 1 2; do
  timeout -k 10 200 python tools/step_ab.py --n 256 --steps 30 --rounds 3 --variants base > gpurun_out/$R/step256_main_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n 256 --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_subswz0.so > gpurun_out/$R/step256_subswz0_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --arch c --n 32 --steps 20 --rounds 3 --variants base > gpurun_out/$R/stepC3_main_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --arch c --n 32 --steps 20 --rounds 3 --variants base --lib ab_libs/libitsd_hip_subswz0.so > gpurun_out/$R/stepC3_subswz0_$r.txt 2>&1 || { echo ab_fail; exit 1; }
done
grep -H best gpurun_out/$R/step*.txt
for f in main subswz0; do
  LIB=""; [ $f = subswz0 ] && LIB="--lib ab_libs/libitsd_hip_subswz0.so"
  timeout -k 10 200 python tools/census.py --n 256 --reps 3 $LIB > gpurun_out/$R/census256_$f.txt 2>&1 || { echo census_fail; exit 1; }
  grep -E "p4_kernel<" gpurun_out/$R/census256_$f.txt | awk -v f=$f '{s[$NF]+=$9} END {for (k in s) printf "%s %s %.4f ms\n", f, k, s[k]}'
done
# (run ai's tail stride A/B in the same call)
R=r05ai; mkdir -p gpurun_out/$R
for L in main tail16; do
  LIB=""; [ $L = tail16 ] && LIB="--lib ab_libs/libitsd_hip_tail16.so"
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES --output-format csv -d gpurun_out/$R/pmc_$L -o run -- python3 tools/census.py --reps 1 --n 256 $LIB > gpurun_out/$R/pmc_$L.log 2>&1 || { echo pmc_fail $L; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for L in ("main", "tail16"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); names = {}
    for fn in glob.glob(f"gpurun_out/r05ai/pmc_{L}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "tail" in r["Kernel_Name"]:
                acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"]); names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0]
    for d, c in acc.items(): print(L, names[d], {k: "%.3g" % v for k, v in c.items()})
PY
for r in 1 2; do
for N in 256 32; do
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base > gpurun_out/$R/step${N}_main_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_tail16.so > gpurun_out/$R/step${N}_tail16_$r.txt 2>&1 || { echo ab_fail; exit 1; }
done
done
grep -H best gpurun_out/$R/step*.txt
for f in main tail16; do
  LIB=""; [ $f = tail16 ] && LIB="--lib ab_libs/libitsd_hip_tail16.so"
  timeout -k 10 200 python tools/census.py --n 256 --reps 3 $LIB > gpurun_out/$R/census256_$f.txt 2>&1 || { echo census_fail; exit 1; }
  grep -E " tail " gpurun_out/$R/census256_$f.txt | head -1 | sed "s/^/$f /"
done
