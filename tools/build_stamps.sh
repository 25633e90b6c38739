#!/bin/bash
# Diagnostic build with in-kernel phase stamps (conv.hip ITSD_STAMPS) and the compile-time ablations
# (ITSD_DIAG): ab_libs/libitsd_hip_stamps.so (ab_libs/ travels to the GPU box; build_diag/ does not).
# Never shipped; tools/stamps.py and tools/census.py --lib load it explicitly.
set -e
cd "$(dirname "$0")/.."
PKG=inference-time-scaling-for-diffusion-models-beyond-scaling-denoising-steps_amd
OUT=${1:-ab_libs}
mkdir -p build_diag "$OUT"
objs=""
for src in $PKG/csrc/*.hip; do
  f=$(basename $src .hip)
  X=""; [ $f = conv ] && X=-fno-slp-vectorize
  /opt/rocm/bin/hipcc $X -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DITSD_STAMPS -DITSD_DIAG -I $PKG/csrc -I include -c $src -o build_diag/$f.o &
  objs="$objs build_diag/$f.o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libitsd_hip_stamps.so $objs
echo $OUT/libitsd_hip_stamps.so
