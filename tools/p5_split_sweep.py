"""Per-op steady-state time of every conv3x3_gn_p5_kernel launch of one forward against its forced K-slice
count (option p5_split), beside the cost model's own choice ("auto"): the data the split cost model
(conv.hip p5_split / p5_plan / p5_combine_cost) is calibrated on. Measurement tool, never part of the product.

    python tools/p5_split_sweep.py --n 32 [--splits 0,1,2,3,4,6,8,12,16] [--img 32]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import itsd  # noqa: F401
from itsd import runtime as rt
from itsd.arch import ARCH_A
from itsd.model import UNet


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--img", type=int, default=32)
    ap.add_argument("--splits", default="0,1,2,3,4,6,8,12,16")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--set", default="", help="itsd_set_option overrides for every column, e.g. p5_c64=2")
    args = ap.parse_args()
    for kv in filter(None, args.set.split("+")):
        k, v = kv.split("=")
        rt.set_option(k, int(v))
    a = ARCH_A
    net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=args.img, precision="bf16",
               weights="gauss").to("cuda:0")
    nat = net.native(args.n)
    x = torch.randn(args.n, 3, args.img, args.img, device="cuda")
    t = torch.full((args.n,), 500, dtype=torch.int32, device="cuda")
    splits = [int(s) for s in args.splits.split(",")]
    ops = nat.profile_ops(x, t)
    p5 = [(i, o) for i, o in enumerate(ops) if "conv3x3_gn_p5_kernel" in o["kernel"]]
    table = {}
    for s in splits:
        rt.set_option("p5_split", s)
        try:
            cur = nat.profile_ops(x, t)  # (the program's op numbering is fixed; folds may change with S)
            kern = {o["op"]: o["kernel"] for o in cur}
            for i, o in p5:
                table[(o["op"], s)] = nat.profile_op(x, t, o["op"], args.reps) * 1e3
                table[(o["op"], "k")] = kern.get(o["op"], "")
        finally:
            rt.set_option("p5_split", 0)
    hdr = " ".join(f"{('auto' if s == 0 else 'S=' + str(s)):>7}" for s in splits)
    print(f"N={args.n} img={args.img} {args.set}: us per launch (steady state, {args.reps} back-to-back)")
    print(f"{'op':>3} {'H':>3} {'M':>6} {'Cout':>5} {'K':>5} {hdr}  best")
    tot = {s: 0.0 for s in splits}
    for i, o in p5:
        row = [table[(o["op"], s)] for s in splits]
        for s, v in zip(splits, row):
            tot[s] += v
        forced = [(v, s) for s, v in zip(splits, row) if s]
        best = f"S={min(forced)[1]}" if forced else ""
        print(f"{o['op']:3d} {o['H']:3d} {o['M']:6d} {o['N']:5d} {o['K']:5d} " + " ".join(f"{v:7.1f}" for v in row)
              + f"  {best} {table.get((o['op'], 'k'), '')}")
    print("sum " + " " * 23 + " ".join(f"{tot[s]:7.1f}" for s in splits))
    if any(splits):
        bestsum = sum(min(table[(o["op"], s)] for s in splits if s) for _, o in p5)
        print(f"per-op best sum {bestsum:.1f} us vs auto {tot[splits[0]] if splits[0] == 0 else float('nan'):.1f} us")


if __name__ == "__main__":
    main()
