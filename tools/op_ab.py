"""Per-op A/B table of one bf16 Arch A forward (census timing: HIP events around every launch)
under several itsd_set_option settings, for the ops of the given kinds.

    python tools/op_ab.py --n 256 --kinds conv --variants base,conv_dbg=16,conv_dbg=2
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import itsd
from itsd import runtime as rt
from itsd.arch import ARCH_A
from itsd.model import UNet

DEFAULTS = {"p5_xl": 3, "splitk": 1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--kinds", default="conv")
    ap.add_argument("--variants", default="base")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    a = ARCH_A
    net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16", weights="gauss").to("cuda:0")
    nat = net.native(args.n)
    x = torch.randn(args.n, 3, 32, 32, device="cuda")
    t = torch.full((args.n,), 500, dtype=torch.int32, device="cuda")
    kinds = set(args.kinds.split(","))
    variants = args.variants.split(",")
    cols = {}
    meta = None
    for v in variants:
        opts = dict(DEFAULTS)
        for kv in v.split("+"):
            if "=" in kv:
                k, val = kv.split("=")
                opts[k] = int(val)
        for k, val in opts.items():
            rt.set_option(k, val)
        best = None
        for _ in range(args.reps):
            ops = nat.profile_ops(x, t)
            ms = [o["ms"] for o in ops]
            best = ms if best is None else [min(p, q) for p, q in zip(best, ms)]
        cols[v] = best
        meta = meta or ops
        for k, val in DEFAULTS.items():
            rt.set_option(k, val)
    print(f"{'#':>3} {'kind':8} {'M':>7} {'N':>5} {'K':>5} {'H':>3} {'ks':>2} " + " ".join(f"{v[:14]:>14}" for v in variants)
          + "  kernel")
    tot = {v: 0.0 for v in variants}
    for i, o in enumerate(meta):
        if o["kind"] not in kinds:
            continue
        for v in variants:
            tot[v] += cols[v][i]
        print(f"{i:3d} {o['kind']:8} {o['M']:7d} {o['N']:5d} {o['K']:5d} {o['H']:3d} {o['ks']:2d} "
              + " ".join(f"{cols[v][i] * 1e3:14.1f}" for v in variants) + f"  {o.get('kernel', '')}")
    print("sum (us)" + " " * 34 + " ".join(f"{tot[v] * 1e3:14.1f}" for v in variants))


if __name__ == "__main__":
    main()
