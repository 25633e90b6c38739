set -o pipefail
# round 5, run j: p4 phase stamps and compile-time ablations after the 16x16x32 MFMA change
R=r05j
mkdir -p gpurun_out/$R
timeout -k 10 300 python tools/stamps.py ab_libs/libitsd_hip_stamps.so all > gpurun_out/$R/stamps256.txt 2>&1 || { echo stamps_fail; tail -5 gpurun_out/$R/stamps256.txt; exit 1; }
timeout -k 10 400 python tools/census.py --n 256 --reps 1 --lib ab_libs/libitsd_hip_diag.so --variants "base,conv_dbg=20480,conv_dbg=36864,conv_dbg=69632,conv_dbg=135168,conv_dbg=151552,conv_dbg=200704,conv_dbg=266240" > gpurun_out/$R/ablate256.txt 2>&1 || { echo ablate_fail; tail -5 gpurun_out/$R/ablate256.txt; exit 1; }
grep variant gpurun_out/$R/ablate256.txt | tail -8
head -30 gpurun_out/$R/stamps256.txt
