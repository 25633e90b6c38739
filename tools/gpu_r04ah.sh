set -o pipefail
R=r04ah
mkdir -p gpurun_out/$R
for v in base small_minks=4 small_minks=8 small_minks=1; do
  timeout -k 10 200 python tools/census.py --n 64 --arch c $( [ $v = base ] || echo --set $v ) > gpurun_out/$R/c64_$v.txt 2>&1 || exit 1
  echo "== C3 $v"; grep -E "^total|conv H[124] |conv H8 " gpurun_out/$R/c64_$v.txt
done
timeout -k 10 400 python tools/step_ab.py --n 32 --variants "base,small_minks=4,small_minks=8" --steps 100 > gpurun_out/$R/step32.txt 2>&1 || exit 1
tail -n 3 gpurun_out/$R/step32.txt
for v in base small_minks=4 small_minks=8; do
  timeout -k 10 300 python tools/leg_time.py --legs C3 $( [ $v = base ] || echo --set $v ) > gpurun_out/$R/c3_$v.txt 2>&1 || exit 1
  echo "$v $(grep -h cand/s gpurun_out/$R/c3_$v.txt)"
done
