#!/bin/bash
# One GPU round trip of the build -> measure loop (run under gpurun from the repo root):
#   tools/gpu_check.sh <out_dir> [pytest selection] -- GPU tests, then per-op census at N = 32 / 64 / 256,
# each step under its own time limit; stops at the first failing step.
out=${1:-gpurun_out/check}; sel=${2:-tests}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest $sel -m gpu -x -v --timeout 200 --timeout-method thread > "$out/tests.log" 2>&1
rc=$?; echo "tests_rc=$rc" >> "$out/tests.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for n in 32 64 256; do
  timeout -k 10 120 python tools/census.py --n $n > "$out/census_$n.txt" 2>&1 || exit $?
done
