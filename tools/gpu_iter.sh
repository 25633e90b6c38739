# One build -> measure iteration on the GPU box: GPU tests (selection $1, default all), census at N = 32 / 64 / 256,
# the p5 launch timeline at N = 32 (stamps build). Stops at the first failing step.
sel=${1:-tests}
timeout -k 10 500 python -u -m pytest $sel -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?; tail -3 gpurun_out/t_all.log; [ $rc -le 1 ] || exit $rc
for n in 32 64 256; do timeout -k 10 100 python tools/census.py --n $n > gpurun_out/c_$n.txt 2>&1 || exit 1; done
timeout -k 10 200 python tools/timeline.py build_diag/libitsd_hip_stamps.so --n 32 2 6 14 22 > gpurun_out/tl_n32.txt 2>&1
