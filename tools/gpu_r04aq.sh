set -o pipefail
R=r04aq
mkdir -p gpurun_out/$R
timeout -k 10 300 python tools/fwd_hash.py > gpurun_out/$R/hash_new.txt 2>&1 || exit 1
timeout -k 10 300 python tools/fwd_hash.py --lib oldlib/libitsd_hip.so > gpurun_out/$R/hash_old.txt 2>&1 || exit 1
tail -n 1 gpurun_out/$R/hash_new.txt gpurun_out/$R/hash_old.txt
for rep in 1 2; do
  for L in new old; do
    LIBARG=$([ $L = old ] && echo "--lib oldlib/libitsd_hip.so" || echo "")
    timeout -k 10 300 python tools/step_ab.py --n 256 --variants base --steps 20 $LIBARG > gpurun_out/$R/s256_${L}_$rep.txt 2>&1 || exit 1
    timeout -k 10 300 python tools/step_ab.py --n 64 --variants base --steps 100 $LIBARG > gpurun_out/$R/s64_${L}_$rep.txt 2>&1 || exit 1
    echo "$L rep$rep: N=256 $(tail -n 1 gpurun_out/$R/s256_${L}_$rep.txt) | N=64 $(tail -n 1 gpurun_out/$R/s64_${L}_$rep.txt)"
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/$R/gpu_tests.log 2>&1 || { echo tests_fail; tail -20 gpurun_out/$R/gpu_tests.log; exit 1; }
tail -n 2 gpurun_out/$R/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$R/smoke.log 2>&1 && tail -n 1 gpurun_out/$R/smoke.log
