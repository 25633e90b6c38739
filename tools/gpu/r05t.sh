set -o pipefail
# round 5, run t: the 8x8 statistics-free convs on conv_small where conv_pipe's 128-tile grid leaves its last round
# part-empty (small_8x8 = 2: N = 256's shortcuts, 384 tiles = 1.5 rounds) vs conv_pipe; and the shipped p4_xcd = 2
R=r05t
mkdir -p gpurun_out/$R
timeout -k 10 300 python tools/step_ab.py --n 256 --steps 30 --rounds 4 --variants "base,small_8x8=2" > gpurun_out/$R/step256_small8.txt 2>&1 || { echo ab_fail; exit 1; }
grep best gpurun_out/$R/step256_small8.txt
timeout -k 10 200 python tools/census.py --n 256 --reps 3 --set small_8x8=2 > gpurun_out/$R/census256_small8_2.txt 2>&1 || { echo census_fail; exit 1; }
timeout -k 10 200 python tools/census.py --n 256 --reps 3 > gpurun_out/$R/census256_base.txt 2>&1 || { echo census_fail; exit 1; }
grep -E " 8  1 " gpurun_out/$R/census256_*.txt | head -12
