"""Phase timeline of attn_block_kernel from the stamps build (tools/build_stamps.sh; kernels.hip ATL(slot):
s_memrealtime, 100 MHz). Never part of the product.

    python tools/attn_timeline.py build_diag/libitsd_hip_stamps.so --n 32
Slots (per wave, µs after the block's entry): 0 entry, 1 group statistics, 2 hn + V^T, 3 scores,
4 softmax, 5 PV, 6 proj + epilogue, 7 exit.
"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import itsd
from itsd import runtime as rt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--n", type=int, default=32)
    args = ap.parse_args()
    rt.LIB_PATH = os.path.abspath(args.lib)
    from itsd.arch import ARCH_A
    from itsd.model import UNet
    a = ARCH_A
    net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16", weights="gauss").to("cuda:0")
    nat = net.native(args.n)
    L = rt.lib()
    x = torch.randn(args.n, 3, 32, 32, device="cuda")
    t = torch.full((args.n,), 500, dtype=torch.int32, device="cuda")
    ops = nat.profile_ops(x, t)
    i = [k for k, o in enumerate(ops) if "attn_block" in o.get("kernel", "")][0]
    ms = nat.profile_op(x, t, ops[i]["op"], reps=3)
    buf = np.zeros(1024 * 128, dtype=np.uint64)
    assert L.itsd_debug_stamps_attn(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong))) == 0
    st = buf.reshape(1024, 16, 8).astype(np.int64)[: min(args.n, 1024)]
    names = ["entry", "group stats", "hn + V^T", "scores", "softmax", "PV", "proj + epilogue", "exit"]
    print(f"op {i} attn_block_kernel N={args.n}: {ms * 1e3:.1f} us/launch")
    for w in (0, 4):
        rel = (st[:, w, :] - st[:, w, :1]) / 100.0
        print(f"  wave {w}: " + "  ".join(f"{n}={rel[:, k].mean():.2f}" for k, n in enumerate(names)))


if __name__ == "__main__":
    main()
