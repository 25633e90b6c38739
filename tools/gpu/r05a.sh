set -o pipefail
# round 5, run a: p4 A-fragment buffer loads (no spills) + XCD tile dealing, against the round-4 build
R=r05a
mkdir -p gpurun_out/$R
timeout -k 10 120 python tools/fwd_hash.py --lib ab_libs/libitsd_r04.so > gpurun_out/$R/hash_r04.txt 2>&1 || { echo hash_old_fail; tail -5 gpurun_out/$R/hash_r04.txt; exit 1; }
timeout -k 10 120 python tools/fwd_hash.py > gpurun_out/$R/hash_new.txt 2>&1 || { echo hash_new_fail; tail -5 gpurun_out/$R/hash_new.txt; exit 1; }
diff <(grep -v amdgpu.ids gpurun_out/$R/hash_r04.txt) <(grep -v amdgpu.ids gpurun_out/$R/hash_new.txt) && echo HASH_SAME || echo HASH_DIFF
timeout -k 10 200 python tools/step_ab.py --n 256 --steps 30 --rounds 3 --variants "base,p4_xcd=1" > gpurun_out/$R/step256_new.txt 2>&1 || { echo ab_fail; tail -5 gpurun_out/$R/step256_new.txt; exit 1; }
timeout -k 10 200 python tools/step_ab.py --n 256 --steps 30 --rounds 3 --variants "base" --lib ab_libs/libitsd_r04.so > gpurun_out/$R/step256_r04.txt 2>&1 || { echo ab_old_fail; exit 1; }
timeout -k 10 200 python tools/step_ab.py --n 256 --steps 30 --rounds 2 --variants "base,p4_xcd=1" > gpurun_out/$R/step256_new2.txt 2>&1 || { echo ab2_fail; exit 1; }
timeout -k 10 200 python tools/census.py --n 256 --reps 3 > gpurun_out/$R/census256_new.txt 2>&1 || { echo census_fail; exit 1; }
timeout -k 10 200 python tools/census.py --n 256 --reps 3 --set p4_xcd=1 > gpurun_out/$R/census256_xcd.txt 2>&1 || { echo census2_fail; exit 1; }
timeout -k 10 200 python tools/census.py --n 256 --reps 3 --lib ab_libs/libitsd_r04.so > gpurun_out/$R/census256_r04.txt 2>&1 || { echo census3_fail; exit 1; }
tail -3 gpurun_out/$R/step256_*.txt
