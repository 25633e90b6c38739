set -o pipefail
R=r04ao
mkdir -p gpurun_out/$R
for v in base conv_dbg=128 conv_dbg=32 conv_dbg=256 conv_dbg=416; do
  timeout -k 10 200 python tools/census.py --n 64 --arch c $( [ $v = base ] || echo --set $v ) > gpurun_out/$R/c64_$v.txt 2>&1 || exit 1
  echo "== $v"; grep -E "^ *(83|85|87|91|93) |conv H1 |conv H2 |^total" gpurun_out/$R/c64_$v.txt
done
