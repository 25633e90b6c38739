set -o pipefail
R=r04ap
mkdir -p gpurun_out/$R
timeout -k 10 300 python tools/fwd_hash.py > gpurun_out/$R/hash_new.txt 2>&1 || exit 1
timeout -k 10 300 python tools/fwd_hash.py --lib oldlib/libitsd_hip.so > gpurun_out/$R/hash_old.txt 2>&1 || exit 1
tail -n 1 gpurun_out/$R/hash_new.txt gpurun_out/$R/hash_old.txt
for rep in 1 2; do
  for L in new old; do
    LIBARG=$([ $L = old ] && echo "--lib oldlib/libitsd_hip.so" || echo "")
    timeout -k 10 300 python tools/step_ab.py --n 32 --variants base --steps 100 $LIBARG > gpurun_out/$R/s32_${L}_$rep.txt 2>&1 || exit 1
    timeout -k 10 300 python tools/census.py --n 64 --arch c $LIBARG > gpurun_out/$R/c64_${L}_$rep.txt 2>&1 || exit 1
    echo "$L rep$rep: N=32 $(tail -n 1 gpurun_out/$R/s32_${L}_$rep.txt) | C3 census $(grep -E '^total' gpurun_out/$R/c64_${L}_$rep.txt) $(grep -E 'conv H1 |conv H2 ' gpurun_out/$R/c64_${L}_$rep.txt | tr -s ' ' | tr '\n' ' ')"
  done
done
