set -o pipefail
R=r04s
mkdir -p gpurun_out/$R
for n in 32 64 128; do
  timeout -k 10 300 python tools/step_ab.py --n $n --variants "base,small_wide=2" --steps 60 > gpurun_out/$R/step$n.txt 2>&1 || exit 1
  tail -2 gpurun_out/$R/step$n.txt
done
