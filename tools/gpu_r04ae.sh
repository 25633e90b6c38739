set -o pipefail
R=r04ae
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 200 --timeout-method thread -k "block_order or convtranspose or split_k" > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed" gpurun_out/$R/tests.log
for v in base wmajor=0 wmajor=2; do
  timeout -k 10 200 python tools/census.py --n 64 --arch c $( [ $v = base ] || echo --set $v ) > gpurun_out/$R/c64_$v.txt 2>&1 || exit 1
  echo "== $v"; grep -E "conv_pipe|^total" gpurun_out/$R/c64_$v.txt | awk '$9>0.03 || /total/'
done
timeout -k 10 400 python tools/leg_time.py --legs C3 > gpurun_out/$R/c3.txt 2>&1 || exit 1
timeout -k 10 400 python tools/leg_time.py --legs C3 --set wmajor=0 > gpurun_out/$R/c3_w0.txt 2>&1 || exit 1
grep -h "cand/s" gpurun_out/$R/c3.txt gpurun_out/$R/c3_w0.txt
timeout -k 10 400 python tools/step_ab.py --n 256 --variants "base,wmajor=0,wmajor=2" --steps 20 > gpurun_out/$R/step256.txt 2>&1 || exit 1
tail -n 4 gpurun_out/$R/step256.txt
