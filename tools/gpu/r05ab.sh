set -o pipefail
# round 5, run ab: the ResBlock 1x1 shortcuts folded into their block2 p5 conv (p5_sc) -- parity, then step A/B at
# N = 32 / 64 / 256, C4 (64 px, N = 16) and C3 (Arch C, N = 32); then run aa's LDS-conflict passes
R=r05ab
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_p5_shortcut.py tests/test_gpu_p5.py tests/test_gpu_attnblock.py -x -v --timeout 250 --timeout-method thread > gpurun_out/$R/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|assert|rel-L2" gpurun_out/$R/tests.log | head -30; exit 1; }
grep -E "passed|failed|folded" gpurun_out/$R/tests.log | tail -12
for N in 32 64 256; do
  timeout -k 10 300 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants "base,p5_sc=0,p5_sc=2" > gpurun_out/$R/step${N}.txt 2>&1 || { echo ab_fail $N; tail -5 gpurun_out/$R/step${N}.txt; exit 1; }
done
timeout -k 10 300 python tools/step_ab.py --n 16 --img 64 --steps 20 --rounds 3 --variants "base,p5_sc=0,p5_sc=2" > gpurun_out/$R/stepC4.txt 2>&1 || { echo ab_fail C4; exit 1; }
timeout -k 10 300 python tools/step_ab.py --arch c --n 32 --steps 20 --rounds 3 --variants "base,p5_sc=0" > gpurun_out/$R/stepC3.txt 2>&1 || { echo ab_fail C3; exit 1; }
grep -H -A4 "best\|variant" gpurun_out/$R/step*.txt | tail -60
timeout -k 10 200 python tools/census.py --n 32 --reps 3 > gpurun_out/$R/census32.txt 2>&1 || { echo census_fail; exit 1; }
tail -16 gpurun_out/$R/census32.txt
bash tools/gpu/r05aa.sh
