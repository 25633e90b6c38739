# A/B of library variants: census at N=32 / 256 for the shipped build and build_diag/libitsd_hip_<v>.so
mkdir -p gpurun_out/ab
for r in 0 1; do for v in base ${VARIANTS:?set VARIANTS}; do for n in 32 256; do
  L=""; [ $v != base ] && L="--lib build_diag/libitsd_hip_$v.so"
  timeout -k 10 100 python tools/census.py --n $n $L > gpurun_out/ab/${v}_${n}_$r.txt 2>&1 || exit 1
done; done; done
