#!/bin/bash
# Host AddressSanitizer build of the C-ABI layer (api.hip) + the validation driver
# tests/asan/abi_validation.cpp -> build_asan/abi_validation. Device code is unchanged (GPU
# sanitizers are not available on this pool): -fsanitize goes to the host side only.
set -e
cd "$(dirname "$0")/.."
PKG=inference-time-scaling-for-diffusion-models-beyond-scaling-denoising-steps_amd
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
OUT=build_asan
mkdir -p $OUT
SAN="-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer"
$HIPCC -O1 -g -std=c++17 -fPIC --offload-arch=gfx950 $SAN -I $PKG/csrc -I include -Wno-unused-result \
  -c $PKG/csrc/api.hip -o $OUT/api_asan.o &
objs=""
for src in $PKG/csrc/*.hip; do  # every device source but api.hip (whose host side is sanitized above)
  f=$(basename $src .hip)
  [ $f = api ] && continue
  X=""; [ $f = conv ] && X=-fno-slp-vectorize
  $HIPCC $X -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I $PKG/csrc -I include -Wno-unused-result \
    -c $src -o $OUT/$f.o &
  objs="$objs $OUT/$f.o"
done
wait
$HIPCC -O1 -g -std=c++17 $SAN -I include -c tests/asan/abi_validation.cpp -o $OUT/abi_validation.o
$HIPCC --offload-arch=gfx950 -fsanitize=address -fno-gpu-sanitize -o $OUT/abi_validation $OUT/abi_validation.o $OUT/api_asan.o \
  $objs
echo $OUT/abi_validation
