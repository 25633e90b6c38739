"""Bit-identity of the XCD-local split-K exchange (option p5_xl) against the write-through one, on Arch A forwards at
several batches (every p5 split form: the shared combine, the two-slice publish-once combine), plus the in-kernel
hand-off status word. Measurement tool, never part of the product.

    python tools/xl_check.py --n 8 16 32 64 128 256
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
    ap.add_argument("--n", type=int, nargs="+", default=[8, 16, 32, 64, 128, 256])
    ap.add_argument("--img", type=int, default=32)
    args = ap.parse_args()
    a = ARCH_A
    net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=args.img, precision="bf16",
               weights="gauss", seed=0).to("cuda:0")
    ok_all = True
    for n in args.n:
        g = torch.Generator().manual_seed(n)
        x = torch.randn(n, 3, args.img, args.img, generator=g).cuda()
        t = torch.randint(0, a.T, (n,), generator=g).cuda()
        outs = []
        for xl in (0, 1, 2, 3, 0, 1, 2, 3):
            rt.set_option("p5_xl", xl)
            e = net(x, t)
            torch.cuda.synchronize()
            st = net.native(n).query("status")
            outs.append((e.clone(), st))
        rt.set_option("p5_xl", 3)
        same = all(torch.equal(outs[0][0], o[0]) for o in outs[1:])
        fin = all(bool(torch.isfinite(o[0]).all()) for o in outs)
        stat = [o[1] for o in outs]
        ok = same and fin and not any(stat)
        ok_all &= ok
        print(f"img {args.img} n={n:4d}: xl bit-identical {same}  finite {fin}  status {stat}  {'OK' if ok else 'FAIL'}",
              flush=True)
    print("ALL OK" if ok_all else "MISMATCH")
    sys.exit(0 if ok_all else 1)


if __name__ == "__main__":
    main()
