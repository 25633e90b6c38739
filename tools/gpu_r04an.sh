set -o pipefail
R=r04an
mkdir -p gpurun_out/$R
timeout -k 10 600 python tools/step_ab.py --n 16 --img 64 --variants "base,small_minks=16,small_minks=32" --steps 60 > gpurun_out/$R/step_c4.txt 2>&1 || exit 1
tail -n 3 gpurun_out/$R/step_c4.txt
timeout -k 10 600 python tools/step_ab.py --n 32 --variants "base,small_minks=16" --steps 100 > gpurun_out/$R/step32.txt 2>&1 || exit 1
tail -n 2 gpurun_out/$R/step32.txt
timeout -k 10 600 python tools/step_ab.py --n 64 --variants "base,small_minks=16" --steps 100 > gpurun_out/$R/step64.txt 2>&1 || exit 1
tail -n 2 gpurun_out/$R/step64.txt
for rep in 1 2; do
for v in base small_minks=16; do
  timeout -k 10 300 python tools/leg_time.py --legs C3 $( [ $v = base ] || echo --set $v ) > gpurun_out/$R/c3_${v}_$rep.txt 2>&1 || exit 1
  echo "$v $(grep -h cand/s gpurun_out/$R/c3_${v}_$rep.txt)"
done
done
