#!/bin/bash
# Diagnostic build (never shipped): hipcc -DITSD_DIAG compiles the superseded fused-conv generations
# (conv_diag.inc: wide / reg / ws / pws, conv_pipe_wide) and the compile-time ablations of
# conv3x3_gn_p4_kernel into build_diag/libitsd_hip_diag.so; load it with ITSD_LIB=... for A/B runs.
# Extra hipcc flags (e.g. -DITSD_STAMPS) come from $ITSD_DIAG_FLAGS.
set -e
cd "$(dirname "$0")/.."
PKG=inference-time-scaling-for-diffusion-models-beyond-scaling-denoising-steps_amd
mkdir -p build_diag
for f in api conv kernels; do
  X=""; [ $f = conv ] && X=-fno-slp-vectorize
  /opt/rocm/bin/hipcc $X -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DITSD_DIAG $ITSD_DIAG_FLAGS -I $PKG/csrc -I include \
    -c $PKG/csrc/$f.hip -o build_diag/diag_$f.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build_diag/libitsd_hip_diag.so build_diag/diag_api.o \
  build_diag/diag_conv.o build_diag/diag_kernels.o
echo build_diag/libitsd_hip_diag.so
