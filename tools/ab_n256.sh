# census A/B at N = 256 and 32: the shipped library vs build_diag/libitsd_hip_$V.so, two interleaved rounds
mkdir -p gpurun_out/ab
for r in 0 1; do for v in base $V; do for n in 256 32; do
  L=""; [ $v != base ] && L="--lib build_diag/libitsd_hip_$v.so"
  timeout -k 10 100 python tools/census.py --n $n $L > gpurun_out/ab/${v}_${n}_$r.txt 2>&1 || exit 1
done; done; done
