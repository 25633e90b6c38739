"""Arch C fp32 forward vs the oracle per image at several batch sizes and build options (diagnostic).
Measurement / debug tool, never part of the product.

    python tools/fp32_archc_check.py [--n 2,64] [--variants base,tap_prune=0+down_merge=0]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from oracle import ref_cpu as R
from itsd import runtime as rt
from itsd.arch import ARCH_C
from itsd.model import CondUNet
from itsd.weights import synthetic_state_dict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="2,64")
    ap.add_argument("--variants", default="base")
    ap.add_argument("--precision", default="fp32")
    args = ap.parse_args()
    a = ARCH_C
    sd = synthetic_state_dict(a, 0)
    for n in [int(v) for v in args.n.split(",")]:
        gen = torch.Generator().manual_seed(641)
        xc = torch.randn(n, 3, 32, 32, generator=gen)
        tc = torch.randint(0, a.T, (n,), generator=gen)
        lab = torch.cat([torch.arange(n // 2) % 10 + 1, torch.zeros(n - n // 2, dtype=torch.long)])
        idx = sorted(set([0, n // 2 - 1, n // 2, n - 1]))
        with torch.no_grad():
            ref = R.unet_forward(sd, xc[idx], tc[idx], a.ch, a.ch_mult, a.attn, a.num_res_blocks, labels=lab[idx],
                                 cfg=True)
        for var in args.variants.split(","):
            opts = {}
            if var != "base":
                for kv in var.split("+"):
                    k, v = kv.split("=")
                    opts[k] = int(v)
            for k, v in opts.items():
                rt.set_option(k, v)
            try:
                net = CondUNet(a.T, a.num_labels, a.ch, a.ch_mult, a.num_res_blocks, 0.0, img_size=32,
                               precision=args.precision)
                net.load_state_dict(sd)
                net = net.to("cuda:0")
                eps = net(xc.cuda(), tc.cuda(), lab.cuda()).float().cpu()
            finally:
                for k in opts:
                    rt.set_option(k, 1)
            d = [(eps[i] - ref[k]).abs().max().item() for k, i in enumerate(idx)]
            print(f"n={n} {var}: max|d| per image {idx}: " + " ".join(f"{v:.2e}" for v in d), flush=True)
            del net
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
