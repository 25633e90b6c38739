set -o pipefail
R=r04ad
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 200 --timeout-method thread -k "convtranspose or subpixel or subpix or small_8x8 or small_wide" > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed|rel-L2|bit-identical" gpurun_out/$R/tests.log
for v in base convt_prune=0; do
  timeout -k 10 200 python tools/census.py --n 64 --arch c $( [ $v = base ] || echo --set $v ) > gpurun_out/$R/c64_$v.txt 2>&1 || exit 1
  echo "== $v"; grep -E "384>|^ *(27|134|145) |^total" gpurun_out/$R/c64_$v.txt
done
timeout -k 10 400 python tools/leg_time.py --legs C3,C4 > gpurun_out/$R/legs.txt 2>&1 || exit 1
grep -h "cand/s" gpurun_out/$R/legs.txt
