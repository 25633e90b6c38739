set -o pipefail
# round 5, run c: p4 phase stamps (diagnostic build) of every fused conv launch at N = 256 and the
# compile-time ablations of p4<32> (conv_dbg 4096 | AB << 13) after the A-fragment buffer loads
R=r05c
mkdir -p gpurun_out/$R
timeout -k 10 300 python tools/stamps.py ab_libs/libitsd_hip_stamps.so all > gpurun_out/$R/stamps256.txt 2>&1 || { echo stamps_fail; tail -5 gpurun_out/$R/stamps256.txt; exit 1; }
timeout -k 10 400 python tools/census.py --n 256 --reps 1 --lib ab_libs/libitsd_hip_diag.so --variants "base,conv_dbg=20480,conv_dbg=36864,conv_dbg=69632,conv_dbg=135168,conv_dbg=151552,conv_dbg=266240" > gpurun_out/$R/ablate256.txt 2>&1 || { echo ablate_fail; tail -5 gpurun_out/$R/ablate256.txt; exit 1; }
grep variant gpurun_out/$R/ablate256.txt | tail -7
for N in 256 32 64; do
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base > gpurun_out/$R/step${N}_new.txt 2>&1 || { echo ab_fail; exit 1; }
  timeout -k 10 200 python tools/step_ab.py --n $N --steps 30 --rounds 3 --variants base --lib ab_libs/libitsd_r04.so > gpurun_out/$R/step${N}_r04.txt 2>&1 || { echo ab_old_fail; tail -3 gpurun_out/$R/step${N}_r04.txt; exit 1; }
done
grep -h best gpurun_out/$R/step*.txt
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { echo bench_fail; tail -5 gpurun_out/$R/bench.err; exit 1; }
tail -c 400 gpurun_out/$R/bench.json
