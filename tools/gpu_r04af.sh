set -o pipefail
R=r04af
mkdir -p gpurun_out/$R
for v in base conv_variant=3 conv_variant=0; do
  timeout -k 10 200 python tools/census.py --n 64 --arch c $( [ $v = base ] || echo --set $v ) > gpurun_out/$R/c64_$v.txt 2>&1 || exit 1
  echo "== $v"; grep -E "conv_pipe|^total" gpurun_out/$R/c64_$v.txt | awk '$9>0.03 || /total/'
done
