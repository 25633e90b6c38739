# p5 K-loop ablations (diagnostic builds, tools/build_variant.sh abN -DITSD_DIAG -DITSD_STAMPS -DP5_AB=N):
# timelines at N = 32 of the stamps build and of the no-A (8) / no-B (16) / neither (24) variants
mkdir -p gpurun_out/abl
for v in ${VARIANTS:-stamps ab8 ab16 ab24}; do
  timeout -k 10 120 python tools/timeline.py build_diag/libitsd_hip_$v.so --n ${N:-32} ${OPS:-2 22} > gpurun_out/abl/$v.txt 2>&1 || exit 1
done
