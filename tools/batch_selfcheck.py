"""Batch independence of the CFG forward (diagnostic): eps of every image of an n-image batch
against the same image run alone (n = 1), fp32. Debug tool, never part of the product.

    python tools/batch_selfcheck.py [--n 64] [--arch c|a] [--set key=val+...]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from itsd import runtime as rt
from itsd.arch import ARCH_A, ARCH_C
from itsd.model import CondUNet, UNet
from itsd.weights import synthetic_state_dict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="64")
    ap.add_argument("--arch", default="c")
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--set", default="")
    args = ap.parse_args()
    for kv in filter(None, args.set.split("+")):
        k, v = kv.split("=")
        rt.set_option(k, int(v))
    a = ARCH_C if args.arch == "c" else ARCH_A
    sd = synthetic_state_dict(a, 0)
    if a.cfg:
        net = CondUNet(a.T, a.num_labels, a.ch, a.ch_mult, a.num_res_blocks, 0.0, img_size=32, precision=args.precision)
    else:
        net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=32, precision=args.precision)
    net.load_state_dict(sd)
    net = net.to("cuda:0")
    for n in [int(v) for v in args.n.split(",")]:
        gen = torch.Generator().manual_seed(641)
        x = torch.randn(n, 3, 32, 32, generator=gen).cuda()
        t = torch.randint(0, a.T, (n,), generator=gen).cuda()
        lab = torch.cat([torch.arange(n // 2) % 10 + 1, torch.zeros(n - n // 2, dtype=torch.long)]).cuda()
        run = (lambda xx, tt, ll: net(xx, tt, ll)) if a.cfg else (lambda xx, tt, ll: net(xx, tt))
        eps = run(x, t, lab).float().cpu()
        d = []
        for i in range(n):
            e1 = run(x[i:i + 1], t[i:i + 1], lab[i:i + 1]).float().cpu()
            d.append((eps[i] - e1[0]).abs().max().item())
        bad = [i for i in range(n) if d[i] > 1e-4]
        print(f"n={n}: max|batch - single| {max(d):.2e}; images > 1e-4: {bad}", flush=True)
        print("  " + " ".join(f"{v:.1e}" for v in d), flush=True)


if __name__ == "__main__":
    main()
