#!/bin/bash
# Diagnostic variant of the library with extra compile definitions (A/B measurements; never shipped):
#   tools/build_variant.sh <name> -DFOO=1 ...  ->  ab_libs/libitsd_hip_<name>.so (ab_libs/ travels to the
# GPU box with the snapshot; objects stay in build_diag/<name>/, which does not).
# Stale objects are deleted first and every compile's exit status is checked, so a failed compile
# can never link an object of an earlier build into the variant.
set -e
cd "$(dirname "$0")/.."
PKG=inference-time-scaling-for-diffusion-models-beyond-scaling-denoising-steps_amd
name=$1; shift
mkdir -p build_diag/$name ab_libs
rm -f build_diag/$name/*.o ab_libs/libitsd_hip_$name.so
pids=()
objs=()
for src in $PKG/csrc/*.hip; do
  f=$(basename $src .hip)
  X=""; [ $f = conv ] && X=-fno-slp-vectorize
  /opt/rocm/bin/hipcc $X -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -I $PKG/csrc -I include -c $src -o build_diag/$name/$f.o &
  pids+=($!)
  objs+=(build_diag/$name/$f.o)
done
for p in "${pids[@]}"; do wait "$p" || { echo "compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ab_libs/libitsd_hip_$name.so "${objs[@]}"
echo ab_libs/libitsd_hip_$name.so
