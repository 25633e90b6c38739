"""Time bench.py's per-GPU legs (C3 CFG / C4 64 px / C5 T=3000) alone, with their census roofline.
Measurement tool, never part of the product.

    python tools/leg_time.py [--legs C3,C4,C5] [--set key=val+key=val]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
import itsd
from itsd import runtime as rt
from itsd.arch import ARCH_A, ARCH_C
from itsd.model import CondUNet, UNet


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--legs", default="C3")
    ap.add_argument("--set", default="")
    args = ap.parse_args()
    for kv in filter(None, args.set.split("+")):
        k, v = kv.split("=")
        rt.set_option(k, int(v))
    dev = torch.device("cuda:0")
    a, c = ARCH_A, ARCH_C
    make = {
        "C3": lambda: bench.leg("C3", lambda: CondUNet(c.T, c.num_labels, c.ch, c.ch_mult, c.num_res_blocks, 0.0,
                                                       img_size=32, precision="bf16", weights="gauss", seed=0,
                                                       device=dev), 32, 32, 1000, 50, cfg=True, workload="C3"),
        "C4": lambda: bench.leg("C4", lambda: UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=64,
                                                   precision="bf16", weights="gauss", seed=0, device=dev),
                                16, 64, 1000, 50, cfg=False, workload="C4"),
        "C5": lambda: bench.leg("C5", lambda: UNet(3000, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=32,
                                                   precision="bf16", weights="gauss", seed=0, device=dev),
                                128, 32, 3000, 100, cfg=False, workload="C5"),
    }
    for name in args.legs.split(","):
        r = make[name]()
        roof = r.get("roofline", {})
        print(f"{name}: {r['value']:.4f} cand/s/GPU  {r['ms_per_step']:.3f} ms/step  "
              f"dominant {roof.get('kernel', '?')} frac {roof.get('frac', float('nan')):.4f}", flush=True)


if __name__ == "__main__":
    main()
