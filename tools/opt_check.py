"""eps of one bf16 Arch A forward under itsd_set_option overrides vs the defaults (relative L2),
plus the oracle-free determinism check (two runs of each variant bit-identical).

    python tools/opt_check.py --n 8,256 small_conv=0 p4_w=3
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="8,256")
    ap.add_argument("variants", nargs="+", help="'+'-joined key=value sets")
    args = ap.parse_args()
    a = ARCH_A
    net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16", weights="gauss").to("cuda:0")
    for n in [int(v) for v in args.n.split(",")]:
        g = torch.Generator().manual_seed(n)
        x = torch.randn(n, 3, 32, 32, generator=g).cuda()
        t = torch.randint(0, 1000, (n,), generator=g).cuda()
        base = net(x, t).float()
        for v in args.variants:
            kv = [p.split("=") for p in v.split("+")]
            old = {}
            for k, val in kv:
                rt.set_option(k, int(val))
            e1 = net(x, t).float()
            e2 = net(x, t).float()
            rel = ((e1 - base).norm() / base.norm()).item()
            print(f"n={n} {v}: rel-L2 vs default {rel:.3e}, deterministic {torch.equal(e1, e2)}", flush=True)
            for k, val in kv:
                rt.set_option(k, {"conv_dbg": 0, "p4_w": 7, "small_conv": 1, "attn_aq": 0, "attn_cs": 0}[k])


if __name__ == "__main__":
    main()
