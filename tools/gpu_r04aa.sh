set -o pipefail
R=r04aa
mkdir -p gpurun_out/$R
for v in base small_8x8=0 subpix_split=0 small_conv=0 p5=2; do
  timeout -k 10 200 python tools/census.py --n 64 --arch c $( [ $v = base ] || echo --set $v ) > gpurun_out/$R/c64_$v.txt 2>&1 || exit 1
  echo "== $v"; grep -E "^ *(27|41|134|135|145|146) |^total" gpurun_out/$R/c64_$v.txt
done
