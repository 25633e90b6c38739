set -o pipefail
R=r04n
mkdir -p gpurun_out/$R
timeout -k 10 300 python tools/step_ab.py --n 32 --variants "base" --steps 100 > gpurun_out/$R/step32_default.txt 2>&1 || exit 1
tail -1 gpurun_out/$R/step32_default.txt
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python tools/step_ab.py --n 32 --variants "base" --steps 100 > gpurun_out/$R/step32_devkernarg.txt 2>&1 || exit 1
tail -1 gpurun_out/$R/step32_devkernarg.txt
timeout -k 10 300 python tools/step_ab.py --n 256 --variants "base" --steps 30 > gpurun_out/$R/step256_default.txt 2>&1 || exit 1
tail -1 gpurun_out/$R/step256_default.txt
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python tools/step_ab.py --n 256 --variants "base" --steps 30 > gpurun_out/$R/step256_devkernarg.txt 2>&1 || exit 1
tail -1 gpurun_out/$R/step256_devkernarg.txt
timeout -k 10 300 python tools/step_ab.py --n 32 --variants "base" --steps 100 > gpurun_out/$R/step32_default2.txt 2>&1 || exit 1
tail -1 gpurun_out/$R/step32_default2.txt
