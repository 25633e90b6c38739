set -o pipefail
# round 5, run u: the one-token AttnBlock fold (Arch C's 1x1 level): parity, C3 census and step A/B (attn_s1 = 1 vs 0)
R=r05u
mkdir -p gpurun_out/$R
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_configs.py -k "one_token or C3 or cfg" -x -v -s --timeout 300 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert|rel-L2" gpurun_out/$R/tests.log | head -20; exit 1; }
grep -E "passed|failed|one-token|folded" gpurun_out/$R/tests.log | tail -4
for r in 1 2; do
  timeout -k 10 200 python tools/step_ab.py --arch c --n 32 --steps 20 --rounds 2 --variants base > gpurun_out/$R/stepC3_fold_$r.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --arch c --n 32 --steps 20 --rounds 2 --variants base --create-set attn_s1=0 > gpurun_out/$R/stepC3_nofold_$r.txt 2>&1 || { echo ab_fail; exit 1; }
done
grep -H best gpurun_out/$R/step*.txt
timeout -k 10 200 python tools/census.py --arch c --n 64 --reps 3 > gpurun_out/$R/censusC3_fold.txt 2>&1 || { echo census_fail; exit 1; }
grep -E "launches" gpurun_out/$R/censusC3_fold.txt | head -20
