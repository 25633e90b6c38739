#!/bin/bash
# Diagnostic variant of the library with extra compile definitions (A/B measurements; never shipped):
#   tools/build_variant.sh <name> -DFOO=1 ...  ->  build_diag/libitsd_hip_<name>.so
set -e
cd "$(dirname "$0")/.."
PKG=inference-time-scaling-for-diffusion-models-beyond-scaling-denoising-steps_amd
name=$1; shift
mkdir -p build_diag/$name
for f in api conv kernels; do
  X=""; [ $f = conv ] && X=-fno-slp-vectorize
  /opt/rocm/bin/hipcc $X -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -I $PKG/csrc -I include -c $PKG/csrc/$f.hip -o build_diag/$name/$f.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build_diag/libitsd_hip_$name.so build_diag/$name/api.o build_diag/$name/conv.o build_diag/$name/kernels.o
echo build_diag/libitsd_hip_$name.so
