set -o pipefail
R=r04ag
mkdir -p gpurun_out/$R
for v in base p5_split=2 p5_split=4 p5_split=6 p5_split=8; do
  timeout -k 10 200 python tools/census.py --n 64 --arch c $( [ $v = base ] || echo --set $v ) > gpurun_out/$R/c64_$v.txt 2>&1 || exit 1
  echo "== C3 $v"; grep -E "^total|convgn H" gpurun_out/$R/c64_$v.txt
done
for v in base p5_split=2 p5_split=4 p5_split=8; do
  timeout -k 10 200 python tools/census.py --n 16 --img 64 $( [ $v = base ] || echo --set $v ) > gpurun_out/$R/c4_$v.txt 2>&1 || exit 1
  echo "== C4 $v"; grep -E "^total|convgn H" gpurun_out/$R/c4_$v.txt
done
