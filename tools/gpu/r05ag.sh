set -o pipefail
# round 5, run ag: conv3x3_gn_p5_kernel's per-level halo swizzle at W <= 16 (main) vs (h >> 1) & 7 (p5swz0 build):
# parity, SQ_LDS_BANK_CONFLICT per p5 instantiation, step A/B at N = 32 / 64 / 256, census p5 times at N = 256 / 32
R=r05ag
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_p5.py tests/test_gpu_p5_shortcut.py tests/test_gpu_attnblock.py tests/test_gpu_bench_configs.py -x -q --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/$R/tests.log | tail -2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in main p5swz0; do
  LIB=""; [ $L = p5swz0 ] && LIB="--lib ab_libs/libitsd_hip_p5swz0.so"
  for N in 256 32; do
    timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES --output-format csv -d gpurun_out/$R/pmc_${L}_$N -o run -- python3 tools/census.py --reps 1 --n $N $LIB > gpurun_out/$R/pmc_${L}_$N.log 2>&1 || { echo pmc_fail $L; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections
for L in ("main", "p5swz0"):
  for N in (256, 32):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); names = {}
    for fn in glob.glob(f"gpurun_out/r05ag/pmc_{L}_{N}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "conv3x3_gn_p5_kernel" in r["Kernel_Name"]:
                acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"]); names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for d, c in acc.items():
        for k, v in c.items(): per[names[d]][k].append(v)
    for n, c in sorted(per.items()):
        print(L, N, n, len(c["SQ_LDS_BANK_CONFLICT"]), {k: "%.3g" % (sum(v) / len(v)) for k, v in c.items()})
PY
for r in 1 2; do
for N in 256 32 64; do
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base > gpurun_out/$R/step${N}_main_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_p5swz0.so > gpurun_out/$R/step${N}_p5swz0_$r.txt 2>&1 || { echo ab_fail; exit 1; }
done
done
grep -H best gpurun_out/$R/step*.txt
for N in 256 32; do
for f in main p5swz0; do
  LIB=""; [ $f = p5swz0 ] && LIB="--lib ab_libs/libitsd_hip_p5swz0.so"
  timeout -k 10 200 python tools/census.py --n $N --reps 3 $LIB > gpurun_out/$R/census${N}_$f.txt 2>&1 || { echo census_fail; exit 1; }
  grep -E "p5_kernel<" gpurun_out/$R/census${N}_$f.txt | awk -v f="$f $N" '{s[$NF]+=$9} END {for (k in s) printf "%s %s %.4f ms\n", f, k, s[k]}'
done
done
