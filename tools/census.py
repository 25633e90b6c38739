"""Per-launch census of one UNet forward on the GPU (HIP events around every launch).

    python tools/census.py [--n 256] [--precision bf16] [--json out.json]
"""
import argparse
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import itsd

CONV_KINDS = ("conv", "convgn", "convgnw", "convgnw4")
from itsd.arch import ARCH_A, ARCH_C
from itsd.model import CondUNet, UNet


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--img", type=int, default=32, help="image size (64: the C4 leg's ImageNet-64 shape)")
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--arch", default="a", help="a: Arch A UNet; c: Arch C CondUNet (the C3 leg; --n is the guided batch 2N)")
    ap.add_argument("--json", default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="", help="comma list of conv_variant values to A/B")
    ap.add_argument("--fuse-gn", type=int, default=1, help="fused GroupNorm+SiLU+conv3x3 in ResBlocks")
    ap.add_argument("--io-mfma", type=int, default=1, help="bf16 head/tail on MFMA (tail GroupNorm fused)")
    ap.add_argument("--lib", default="", help="another build of libitsd_hip.so (diagnostic variants)")
    ap.add_argument("--set", default="", help="itsd_set_option overrides for the final table, e.g. gn_wide=1+conv_dbg=2")
    args = ap.parse_args()
    from itsd import runtime as rt
    if args.lib:
        rt.LIB_PATH = os.path.abspath(args.lib)
    rt.set_option("fuse_gn", args.fuse_gn)
    rt.set_option("io_mfma", args.io_mfma)
    if args.arch == "c":
        c = ARCH_C
        net = CondUNet(c.T, c.num_labels, c.ch, c.ch_mult, c.num_res_blocks, 0.0, img_size=args.img,
                       precision=args.precision, weights="gauss")
    else:
        a = ARCH_A
        net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=args.img, precision=args.precision,
                   weights="gauss")
    net.to("cuda:0")
    nat = net.native(args.n)
    x = torch.randn(args.n, 3, args.img, args.img, device="cuda")
    t = torch.full((args.n,), 500, dtype=torch.int32, device="cuda")
    if args.variants:
        # each variant: '+'-joined itsd_set_option key=value pairs, e.g.
        # "base", "small_conv=0", "conv_variant=2+splitk=0", "conv_dbg=19"
        defaults = {"conv_variant": 2, "splitk": 1, "small_conv": 1, "gn_wide": 1,
                    "p4_w": 7, "p5": 1, "p5_split": 0, "gn_fold": 1,
                    "small_wide": 1, "small_8x8": 1, "subpix_split": 1, "conv1x1": 1, "attn_wide": 1,
                    "attn_wide_nq": 1, "attn_split": 1, "p4_sub": 1, "p4_plain": 1, "splitk_inl": 1, "convt_prune": 1, "p5_dist": 1, "p5_pub": 1, "small_gn": 1}
        # (diagnostic keys -- conv_dbg, small_minks, ... -- only where a variant names them: the shipped build refuses them)
        for rnd in range(3):
            for v in args.variants.split(","):
                opts = dict(defaults)
                for kv in v.split("+"):
                    if "=" in kv:
                        k, val = kv.split("=")
                        opts[k] = int(val)
                for k, val in opts.items():
                    rt.set_option(k, val)
                ops = nat.profile_ops(x, t)
                conv = [o for o in ops if o["kind"] in CONV_KINDS]
                by = defaultdict(lambda: [0.0, 0.0])
                for o in conv:
                    by[o["H"]][0] += o["ms"]
                    by[o["H"]][1] += o["flops"]
                print(f"round {rnd} variant {v}: conv {sum(o['ms'] for o in conv):.3f} ms total {sum(o['ms'] for o in ops):.3f} ms | "
                      + " ".join(f"H{h}:{m:.3f}ms/{f / m / 1e9:.0f}TF" for h, (m, f) in sorted(by.items())))
        for k, val in defaults.items():
            rt.set_option(k, val)
    for kv in filter(None, args.set.split("+")):
        k, val = kv.split("=")
        rt.set_option(k, int(val))
    for _ in range(args.reps):
        ops = nat.profile_ops(x, t)
    tot = sum(o["ms"] for o in ops)
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    print(f"{'#':>3} {'kind':5} {'M':>7} {'N':>5} {'K':>5} {'H':>3} {'ks':>2} {'s/u':>3} {'ms':>8} {'TF/s':>7}")
    for i, o in enumerate(ops):
        tf = o["flops"] / (o["ms"] * 1e-3) / 1e12 if o["ms"] > 0 and o["flops"] > 0 else 0.0
        print(f"{i:3d} {o['kind']:5} {o['M']:7d} {o['N']:5d} {o['K']:5d} {o['H']:3d} {o['ks']:2d} {o['stride_up']:3d} "
              f"{o['ms']:8.4f} {tf:7.1f}  {o.get('kernel', '')}")
        key = o["kind"] if o["kind"] not in CONV_KINDS else f"{o['kind']} H{o['H']}"
        agg[key][0] += 1
        agg[key][1] += o["ms"]
        agg[key][2] += o["flops"]
    print(f"total {tot:.3f} ms")
    for k, (c, m, f) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:10} launches {c:3d}  {m:8.3f} ms ({100 * m / tot:5.1f}%)  "
              f"{(f / (m * 1e-3) / 1e12) if f else 0:7.1f} TF/s")
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(ops, fh)


if __name__ == "__main__":
    main()
