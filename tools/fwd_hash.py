"""Hash of the forward outputs (Arch C 2N=64 guided, Arch A N=32 / 256) for a build given by --lib:
bit-identity checks between two builds run as two processes. Measurement tool, never part of the product.

    python tools/fwd_hash.py [--lib path/to/libitsd_hip.so]
"""
import argparse
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    args = ap.parse_args()
    from itsd import runtime as rt
    if args.lib:
        rt.LIB_PATH = os.path.abspath(args.lib)
    from itsd.arch import ARCH_A, ARCH_C
    from itsd.model import CondUNet, UNet
    from itsd.weights import synthetic_state_dict
    out = []
    for a, n in ((ARCH_C, 64), (ARCH_A, 32), (ARCH_A, 256)):
        if a.cfg:
            net = CondUNet(a.T, a.num_labels, a.ch, a.ch_mult, a.num_res_blocks, 0.0, precision="bf16")
        else:
            net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, precision="bf16")
        net.load_state_dict(synthetic_state_dict(a, 0))
        net.to("cuda:0")
        gen = torch.Generator().manual_seed(77 + n)
        x = torch.randn(n, 3, 32, 32, generator=gen).cuda()
        t = torch.randint(0, a.T, (n,), generator=gen).cuda()
        extra = [torch.cat([torch.arange(n // 2) % 10 + 1, torch.zeros(n - n // 2, dtype=torch.long)]).cuda()] if a.cfg else []
        e = net(x, t, *extra).float().cpu().contiguous()
        out.append(f"{a.kind} n={n}: {hashlib.sha256(e.numpy().tobytes()).hexdigest()[:16]}")
    print(" | ".join(out))


if __name__ == "__main__":
    main()
