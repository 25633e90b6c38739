set -o pipefail
R=r04ai
mkdir -p gpurun_out/$R
timeout -k 10 400 python tools/step_ab.py --n 32 --variants "base,small_minks=4,small_minks=8,small_minks=16" --steps 100 > gpurun_out/$R/step32.txt 2>&1 || exit 1
tail -n 4 gpurun_out/$R/step32.txt
timeout -k 10 400 python tools/step_ab.py --n 64 --variants "base,small_minks=4,small_minks=8,small_minks=16" --steps 100 > gpurun_out/$R/step64.txt 2>&1 || exit 1
tail -n 4 gpurun_out/$R/step64.txt
timeout -k 10 400 python tools/step_ab.py --n 256 --variants "base,small_minks=8" --steps 20 > gpurun_out/$R/step256.txt 2>&1 || exit 1
tail -n 2 gpurun_out/$R/step256.txt
for rep in 1 2; do
for v in base small_minks=4 small_minks=8; do
  timeout -k 10 300 python tools/leg_time.py --legs C3,C4 $( [ $v = base ] || echo --set $v ) > gpurun_out/$R/legs_${v}_$rep.txt 2>&1 || exit 1
  echo "$v $(grep -h cand/s gpurun_out/$R/legs_${v}_$rep.txt | tr '\n' ' ')"
done
done
