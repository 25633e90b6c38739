"""A/B of itsd_set_option settings on the graph-replayed sampler step (the bench's timed path), in one
process, interleaved. Measurement tool, never part of the product.

    python tools/step_ab.py --n 32 --variants "base,sc_side=0" [--steps 50] [--rounds 3]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import itsd
from itsd import runtime as rt
from itsd.arch import ARCH_A
from itsd.diffusion import GaussianDiffusionSampler
from itsd.model import UNet


# the shipped value of every option a variant may touch (a variant's keys are reset to these after it runs)
DEFAULTS = {"gn_fold": 1, "p5": 1, "p5_split": 0, "p5_sc": 1, "splitk_inl": 1, "p4_plain": 1, "splitk": 1, "attn_split": 1,
            "p4_sub": 1, "gn_wide": 1, "small_conv": 1, "conv_variant": 2, "small_wide": 1, "small_8x8": 1,
            "subpix_split": 1, "conv1x1": 1, "attn_wide": 1, "attn_wide_nq": 1, "p4_w": 7, "convt_prune": 1, "small_minks": 8,
            "attn_fuse": 1, "fuse_gn": 1, "conv_dbg": 0, "p4_xcd": 2, "spin_bound": 1 << 22, "p4_c96": 1, "p5_dist": 1, "p5_pub": 1, "small_gn": 1, "p5_xl": 3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--img", type=int, default=32)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="base")
    ap.add_argument("--create-set", default="", help="options set before the UNet is created, e.g. attn_fuse=0")
    ap.add_argument("--lib", default="", help="another build of libitsd_hip.so (A/B of two builds in two processes)")
    ap.add_argument("--arch", default="a", help="a: Arch A; c: the C3 leg (Arch C CondUNet, CFG w=1.8: --n is N, 2N guided)")
    args = ap.parse_args()
    if args.lib:
        rt.LIB_PATH = os.path.abspath(args.lib)
    for kv in filter(None, args.create_set.split("+")):
        k, val = kv.split("=")
        rt.set_option(k, int(val))
    run_kw = {}
    if args.arch == "c":
        from itsd.arch import ARCH_C
        from itsd.diffusion import CondGaussianDiffusionSampler
        from itsd.model import CondUNet
        c = ARCH_C
        net = CondUNet(c.T, c.num_labels, c.ch, c.ch_mult, c.num_res_blocks, 0.0, img_size=args.img, precision="bf16",
                       weights="gauss").to("cuda:0")
        smp = CondGaussianDiffusionSampler(net, 1e-4, 0.028, 1000, w=1.8)
        run_kw["labels"] = (torch.arange(args.n, device="cuda") % 10 + 1).to(torch.int32)
    else:
        a = ARCH_A
        net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=args.img, precision="bf16",
                   weights="gauss").to("cuda:0")
        smp = GaussianDiffusionSampler(net, 1e-4, 0.02, 1000)
    x = torch.randn(args.n, 3, args.img, args.img, device="cuda")
    variants = args.variants.split(",")
    res = {v: [] for v in variants}
    for r in range(args.rounds):
        for v in variants:
            opts = {}
            for kv in v.split("+"):
                if "=" in kv:
                    k, val = kv.split("=")
                    opts[k] = int(val)
            for k, val in opts.items():
                rt.set_option(k, val)
            smp.run(x.clone(), t_begin=999, t_end=999 - 4, seed=1, **run_kw)  # capture + warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            smp.run(x.clone(), t_begin=999, t_end=999 - args.steps + 1, seed=1, **run_kw)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / args.steps
            res[v].append(ms)
            for k in opts:  # back to the default of each option touched
                rt.set_option(k, DEFAULTS[k])
            print(f"round {r} {v}: {ms:.4f} ms/step", flush=True)
    for v in variants:
        print(f"{v}: best {min(res[v]):.4f} ms/step  ({args.n * 1000 / min(res[v]) / 1000 * 1000 / 1000:.2f} cand/s at T=1000)")


if __name__ == "__main__":
    main()
