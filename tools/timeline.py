"""Launch timelines of the fused GroupNorm convs from the stamps build (tools/build_stamps.sh; conv.hip
TL(slot): s_memrealtime, 100 MHz, one clock for every block). Never part of the product.

    python tools/timeline.py build_diag/libitsd_hip_stamps.so --n 32 [op_index ...]

Per op: the launch's last repetition, every block's stamps relative to the earliest block entry (us):
conv3x3_gn_p5_kernel -- MFMA wave 0: 0 entry, 1 after B0, 2 K loop done (last item), 3 split-K combined,
4 epilogue done, 5 exit (the shared-combine form <W, CB, true>: 3 partial stored + arrived, 4 every slice
arrived, 5 combine and epilogue done), 6 first chunk computed, 7 after its barrier; halo wave 4: 0 entry, 1 first item
opened (group statistics), 2 stage 0 emitted, 3 after B0, 4 stage 1 emitted, 6 after its barrier, 5 exit.
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
    ap.add_argument("ops", nargs="*", type=int)
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--kernel", default="conv3x3_gn_p5_kernel")
    ap.add_argument("--set", default="")
    args = ap.parse_intermixed_args()
    rt.LIB_PATH = os.path.abspath(args.lib)
    from itsd.arch import ARCH_A
    from itsd.model import UNet
    a = ARCH_A
    net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16", weights="gauss").to("cuda:0")
    nat = net.native(args.n)
    L = rt.lib()
    for kv in filter(None, args.set.split("+")):
        k, v = kv.split("=")
        rt.set_option(k, int(v))
    x = torch.randn(args.n, 3, 32, 32, device="cuda")
    t = torch.full((args.n,), 500, dtype=torch.int32, device="cuda")
    ops = nat.profile_ops(x, t)
    sel = args.ops or [i for i, o in enumerate(ops) if args.kernel in o.get("kernel", "")]
    for i in sel:
        o = ops[i]
        ms = nat.profile_op(x, t, o["op"], reps=3)
        buf = np.zeros(1024 * 128, dtype=np.uint64)
        assert L.itsd_debug_stamps(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong))) == 0
        st = buf.reshape(1024, 16, 8).astype(np.int64)
        e0 = st[:, 0, 0]
        last = e0.max()
        blk = np.nonzero((e0 > 0) & (e0 > last - 2000))[0]  # this launch's blocks (entries within 20 us)
        st = st[blk]
        base = st[:, 0, 0].min()
        us = lambda v: (v - base) / 100.0
        print(f"op {i:3d} {o['kernel']:28s} M={o['M']} N={o['N']} K={o['K']} H={o['H']}: {ms * 1e3:.1f} us/launch, "
              f"{len(blk)} blocks")
        def row(name, w, s, valid=None):
            v = st[:, w, s]
            m = v > base - 1 if valid is None else valid
            m &= v > 0
            if not m.any():
                print(f"   {name:24s} -")
                return
            u = us(v[m])
            print(f"   {name:24s} n={m.sum():4d}  min {u.min():7.2f}  mean {u.mean():7.2f}  max {u.max():7.2f}")
        simd = st[:, 8:16, 0]
        print("   SIMD of waves 0..7 (first 4 blocks): " + "  ".join("".join(str(int(v)) for v in simd[b]) for b in range(min(4, len(simd)))))
        p4s = buf.reshape(1024, 16, 8)[:, 8:16, 1].astype(np.int64)
        print("   p4 (last launch) SIMD of waves 0..7 (first 4 blocks): " + "  ".join("".join(str(int(v)) for v in p4s[b]) for b in range(4)))
        row("mfma entry", 0, 0)
        row("mfma after B0", 0, 1)
        row("mfma chunk 0 computed", 0, 6)
        row("mfma chunk 0 barrier", 0, 7)
        row("mfma K loop done", 0, 2)
        if ", true>" in o["kernel"]:  # p5's shared combine (DIST): slots 3 / 4 / 5 mark its hand-off
            row("mfma partial + arrived", 0, 3)
            row("mfma all slices arrived", 0, 4)
            row("mfma combine+epi done", 0, 5)
        else:  # last-arriver / publish-once combine (a first arriver skips 3 and 4)
            row("mfma split-K combined", 0, 3)
            row("mfma epilogue done", 0, 4)
            row("mfma exit", 0, 5)
        d_rt = (st[:, 0, 2] - st[:, 0, 1]).astype(np.float64)
        d_mt = (st[:, 1, 2] - st[:, 1, 1]).astype(np.float64)
        ok = (d_rt > 0) & (d_mt > 0)
        if ok.any():
            print(f"   shader clock over the K loop (wave 1 memtime / wave 0 realtime): "
                  f"{np.median(d_mt[ok] / d_rt[ok]) * 0.1:.2f} GHz")
        row("halo entry", 4, 0)
        row("halo kernargs in SGPRs", 4, 7)
        row("halo item 0 opened", 4, 1)
        row("halo stage 0 emitted", 4, 2)
        row("halo after B0", 4, 3)
        row("halo stage 1 emitted", 4, 4)
        row("halo stage 1 barrier", 4, 6)
        row("halo exit", 4, 5)


if __name__ == "__main__":
    main()
