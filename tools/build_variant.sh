#!/bin/bash
# Diagnostic variant of the library with extra compile definitions (A/B measurements; never shipped):
#   tools/build_variant.sh <name> -DFOO=1 ...  ->  build_diag/libitsd_hip_<name>.so
# Stale objects are deleted first and every compile's exit status is checked, so a failed compile
# can never link an object of an earlier build into the variant.
set -e
cd "$(dirname "$0")/.."
PKG=inference-time-scaling-for-diffusion-models-beyond-scaling-denoising-steps_amd
name=$1; shift
mkdir -p build_diag/$name
rm -f build_diag/$name/*.o build_diag/libitsd_hip_$name.so
pids=()
for f in api conv kernels; do
  X=""; [ $f = conv ] && X=-fno-slp-vectorize
  /opt/rocm/bin/hipcc $X -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -I $PKG/csrc -I include -c $PKG/csrc/$f.hip -o build_diag/$name/$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p" || { echo "compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build_diag/libitsd_hip_$name.so build_diag/$name/api.o build_diag/$name/conv.o build_diag/$name/kernels.o
echo build_diag/libitsd_hip_$name.so
