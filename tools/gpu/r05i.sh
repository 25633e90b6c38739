set -o pipefail
# round 5, run i: p4 on 16x16x32 without spills (tb[4] + immediate offsets): every RES form (m16all) and the 32x32
# level only (m16w32) vs 32x32x16 (m32); parity of the all-forms build
R=r05i
mkdir -p gpurun_out/$R
export ITSD_LIB=$PWD/ab_libs/libitsd_hip_m16all.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert" gpurun_out/$R/tests.log | head -20; exit 1; }
tail -1 gpurun_out/$R/tests.log
unset ITSD_LIB
for r in 1 2; do
for v in m32 m16all m16w32; do
  timeout -k 10 200 python tools/step_ab.py --n 256 --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_hip_$v.so > gpurun_out/$R/step256_${v}_$r.txt 2>&1 || { echo ab_fail; exit 1; }
done
done
grep -H best gpurun_out/$R/step*.txt
for v in m32 m16all; do
timeout -k 10 200 python tools/census.py --n 256 --reps 3 --lib ab_libs/libitsd_hip_$v.so > gpurun_out/$R/census256_$v.txt 2>&1 || { echo census_fail; exit 1; }
done
