set -o pipefail
# round 5, run y: current C4 (64 px, N = 16) and N = 32 censuses
R=r05y
mkdir -p gpurun_out/$R
timeout -k 10 200 python tools/census.py --n 16 --img 64 --reps 3 > gpurun_out/$R/censusC4.txt 2>&1 || { echo census_fail; exit 1; }
timeout -k 10 200 python tools/census.py --n 32 --reps 3 > gpurun_out/$R/census32.txt 2>&1 || { echo census_fail; exit 1; }
grep -E "launches" gpurun_out/$R/censusC4.txt | head -16
grep -E "launches" gpurun_out/$R/census32.txt | head -16
