"""Phase shares of the wide fused conv from a diagnostic build (hipcc -DITSD_STAMPS, see
conv.hip: per wave, s_memtime cycles in wait / barrier / weight-DMA issue / MFMA issue /
GN transform, plus prologue, epilogue and total). Never part of the product.

    python tools/stamps.py build_diag/libitsd_hip_stamps.so [op_index ...]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import itsd
from itsd import runtime as rt

rt.LIB_PATH = os.path.abspath(sys.argv[1])
from itsd.arch import ARCH_A
from itsd.model import UNet

N = 256
a = ARCH_A
net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16", weights="gauss").to("cuda:0")
nat = net.native(N)
x = torch.randn(N, 3, 32, 32, device="cuda")
t = torch.full((N,), 500, dtype=torch.int32, device="cuda")
ops = nat.profile_ops(x, t)
L = rt.lib()
names = ["wait", "barrier", "issue", "mma", "transform", "prologue", "epilogue", "total"]
sel = [int(v) for v in sys.argv[2:]] or [i for i, o in enumerate(ops) if o["kind"] in ("convgnw", "convgnw4")][:6]
for i in sel:
    o = ops[i]
    L.itsd_set_option(b"conv_dbg", int(os.environ.get("ITSD_DBG", "0")))
    ms = nat.profile_op(x, t, i, reps=3)
    buf = np.zeros(1024 * 64, dtype=np.uint64)
    assert L.itsd_debug_stamps(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong))) == 0
    st = buf.reshape(1024, 8, 8).astype(np.float64)
    nb = min(1024, (o["M"] // 256) * (o["N"] // 128))
    st = st[:nb]
    tot = st[:, :, 7].mean()
    taps = o["K"] // 64
    print(f"op {i:3d} {o['kind']:8s} M={o['M']} N={o['N']} K={o['K']} H={o['H']}: {ms*1e3:.1f} us/launch, "
          f"block {tot:.0f} memtime ticks, {taps} taps")
    print("   " + "  ".join(f"{n}={st[:, :, k].mean():.0f} ({100*st[:, :, k].mean()/tot:.0f}%)" for k, n in enumerate(names[:7])))
    print("   per tap: " + "  ".join(f"{n}={st[:, :, k].mean()/taps:.0f}" for k, n in enumerate(names[:5])))
    print("   waves (mma share): " + " ".join(f"{100*st[:, w, 3].mean()/tot:.0f}" for w in range(8)))
