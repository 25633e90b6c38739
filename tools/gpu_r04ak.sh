set -o pipefail
R=r04ak
mkdir -p gpurun_out/$R
timeout -k 10 600 python -u -m pytest tests/test_gpu_attnblock.py -v -s --timeout 300 --timeout-method thread > gpurun_out/$R/tests.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed|rel-L2|Error|assert" gpurun_out/$R/tests.log | tail -20
for rep in 1 2; do
for n in 32 256; do
  for cs in attn_fuse=1 attn_fuse=2; do
    timeout -k 10 300 python tools/step_ab.py --n $n --variants base --steps $([ $n = 32 ] && echo 100 || echo 20) --create-set $cs > gpurun_out/$R/step${n}_${cs}_$rep.txt 2>&1 || exit 1
    echo "n=$n $cs $(tail -n 1 gpurun_out/$R/step${n}_${cs}_$rep.txt)"
  done
done
done
timeout -k 10 200 python tools/census.py --n 32 > gpurun_out/$R/c32.txt 2>&1 || exit 1
grep -E " 4 .*(attn|gn)|^total" gpurun_out/$R/c32.txt
