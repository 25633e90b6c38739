"""A/B of the fused GroupNorm conv variants per UNet level: eps of one bf16 forward with
gn_reg=4 (conv3x3_gn_p4_kernel) restricted to the levels in p4_w vs gn_reg=3 (pws)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import itsd
from itsd import runtime as rt
from itsd.arch import ARCH_A
from itsd.model import UNet


def main():
    a = ARCH_A
    net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16", weights="gauss").to("cuda:0")
    for n in [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "8,256").split(",")]:
        g = torch.Generator().manual_seed(n)
        x = torch.randn(n, 3, 32, 32, generator=g).cuda()
        t = torch.randint(0, 1000, (n,), generator=g).cuda()
        rt.set_option("gn_reg", 3)
        base = net(x, t).float()
        for mask in (1, 2, 4, 7):
            rt.set_option("gn_reg", 4)
            rt.set_option("p4_w", mask)
            e = net(x, t).float()
            rel = ((e - base).norm() / base.norm()).item()
            print(f"n={n} p4_w={mask}: rel-L2 vs pws {rel:.3e}", flush=True)
        rt.set_option("gn_reg", 3)
        rt.set_option("p4_w", 7)


if __name__ == "__main__":
    main()
