"""Phase shares of the fused GroupNorm convs from a diagnostic build (tools/build_stamps.sh:
hipcc -DITSD_STAMPS, see conv.hip; per wave, s_memtime cycles). Never part of the product.

    python tools/stamps.py build_diag/libitsd_hip_stamps.so [op_index ...]

conv3x3_gn_p4_kernel (persistent, one MFMA wave per SIMD): MFMA waves 0..3 (chunk compute, barrier
wait, epilogue, total), halo waves 4..7 (stage transform, barrier wait, prologue, total).
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

N = int(os.environ.get("ITSD_N", "256"))
GN_REG = 4  # (the superseded generations 0-3 and their "gn_reg" switch are gone)
a = ARCH_A
net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16", weights="gauss").to("cuda:0")
nat = net.native(N)
x = torch.randn(N, 3, 32, 32, device="cuda")
t = torch.full((N,), 500, dtype=torch.int32, device="cuda")
L = rt.lib()
ops = nat.profile_ops(x, t)
conv_p4 = [i for i, o in enumerate(ops) if o["kind"] in ("convgnw", "convgnw4")]
sel = conv_p4 if sys.argv[2:] == ["all"] else ([int(v) for v in sys.argv[2:]] or conv_p4[:6])
for i in sel:
    o = ops[i]
    L.itsd_set_option(b"conv_dbg", int(os.environ.get("ITSD_DBG", "0")))
    ms = nat.profile_op(x, t, o["op"], reps=3)
    buf = np.zeros(1024 * 128, dtype=np.uint64)
    assert L.itsd_debug_stamps(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong))) == 0
    st = buf.reshape(1024, 16, 8).astype(np.float64)
    nb = min(1024, (o["M"] // 256) * (o["N"] // 128))
    st = st[:nb]
    chunks = o["K"] // (9 * 64)
    if GN_REG in (3, 4):
        NM = 8 if GN_REG == 3 else 4  # MFMA waves; the 4 halo waves follow
        tiles = (o["M"] // 256) * (o["N"] // 128)
        G = min(tiles, 256)
        st = buf.reshape(1024, 16, 8).astype(np.float64)[:G]
        tot = st[:, :NM, 7].mean()
        tpb = tiles / G
        print(f"op {i:3d} {o['kind']:8s} M={o['M']} N={o['N']} K={o['K']} H={o['H']}: {ms*1e3:.1f} us/launch, "
              f"block {tot:.0f} memtime ticks, {tpb:.2f} tiles x {chunks} chunks per block")
        m = st[:, :NM]
        print("   MFMA waves: " + "  ".join(f"{n}={m[:, :, k].mean():.0f} ({100*m[:, :, k].mean()/tot:.0f}%)"
                                           for k, n in ((0, "compute"), (1, "barrier"), (6, "epilogue"))))
        print(f"     per chunk: compute={m[:, :, 0].mean()/(chunks*tpb):.0f}  barrier={m[:, :, 1].mean()/(chunks*tpb):.0f}"
              f"  epilogue/tile={m[:, :, 6].mean()/tpb:.0f}")
        h = st[:, NM:NM + 4]
        print("   halo waves: " + "  ".join(f"{n}={h[:, :, k].mean():.0f} ({100*h[:, :, k].mean()/tot:.0f}%)"
                                           for k, n in ((3, "transform"), (1, "barrier"), (5, "prologue"))))
        print(f"     per stage: transform={h[:, :, 3].mean()/(chunks*tpb):.0f}")
    elif GN_REG == 2:
        tot = st[:, :8, 7].mean()
        print(f"op {i:3d} {o['kind']:8s} M={o['M']} N={o['N']} K={o['K']} H={o['H']}: {ms*1e3:.1f} us/launch, "
              f"block {tot:.0f} memtime ticks, {chunks} chunks")
        m = st[:, :8]
        print("   MFMA waves: " + "  ".join(f"{n}={m[:, :, k].mean():.0f} ({100*m[:, :, k].mean()/tot:.0f}%)"
                                           for k, n in ((0, "compute"), (1, "barrier"), (5, "prologue"), (6, "epilogue"))))
        print(f"     per chunk: compute={m[:, :, 0].mean()/chunks:.0f}  barrier={m[:, :, 1].mean()/(chunks+2):.0f}")
        h = st[:, 8:12]
        print("   halo waves: " + "  ".join(f"{n}={h[:, :, k].mean():.0f} ({100*h[:, :, k].mean()/tot:.0f}%)"
                                           for k, n in ((3, "staging"), (1, "barrier"), (5, "chunk0"), (6, "output"))))
        if chunks > 1:
            print(f"     per chunk: staging={h[:, :, 3].mean()/(chunks-1):.0f}")
    else:
        names = ["wait", "barrier", "issue", "mma", "transform", "prologue", "epilogue", "total"]
        st = st[:, :8]
        tot = st[:, :, 7].mean()
        taps = o["K"] // 64
        print(f"op {i:3d} {o['kind']:8s} M={o['M']} N={o['N']} K={o['K']} H={o['H']}: {ms*1e3:.1f} us/launch, "
              f"block {tot:.0f} memtime ticks, {taps} taps")
        print("   " + "  ".join(f"{n}={st[:, :, k].mean():.0f} ({100*st[:, :, k].mean()/tot:.0f}%)" for k, n in enumerate(names[:7])))
        print("   per tap: " + "  ".join(f"{n}={st[:, :, k].mean()/taps:.0f}" for k, n in enumerate(names[:5])))
