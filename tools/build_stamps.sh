#!/bin/bash
# Diagnostic build with in-kernel phase stamps (conv.hip ITSD_STAMPS): build_diag/libitsd_hip_stamps.so.
# Never shipped; tools/stamps.py loads it explicitly.
set -e
cd "$(dirname "$0")/.."
PKG=inference-time-scaling-for-diffusion-models-beyond-scaling-denoising-steps_amd
mkdir -p build_diag
for f in api conv kernels; do
  X=""; [ $f = conv ] && X=-fno-slp-vectorize
  /opt/rocm/bin/hipcc $X -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DITSD_STAMPS -DITSD_DIAG -I $PKG/csrc -I include -c $PKG/csrc/$f.hip -o build_diag/$f.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build_diag/libitsd_hip_stamps.so build_diag/api.o build_diag/conv.o build_diag/kernels.o
echo build_diag/libitsd_hip_stamps.so
