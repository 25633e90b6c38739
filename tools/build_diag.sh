#!/bin/bash
# Diagnostic build (never shipped): hipcc -DITSD_DIAG compiles the compile-time ablations of
# conv3x3_gn_p4_kernel (conv_dbg 4096 | AB << 13) and the p5 K-loop ablation switches into
# ab_libs/libitsd_hip_diag.so; load it with ITSD_LIB=... (or --lib) for A/B runs.
# Extra hipcc flags (e.g. -DITSD_STAMPS) come from $ITSD_DIAG_FLAGS.
exec "$(dirname "$0")/build_variant.sh" diag -DITSD_DIAG $ITSD_DIAG_FLAGS
