"""Library-GEMM reference points for the UNet's conv shapes (measurement only).

For every distinct (M, N, K) of a census (tools/census.py --json), times torch.mm of
bf16 [M, K] x [K, N] (hipBLASLt) on the GPU: the rate a plain library GEMM of the same
shape reaches without the implicit im2col, the fused epilogue or the GroupNorm.

    python tools/gemm_ceiling.py census.json
"""
import json
import sys

import torch


def main():
    ops = json.load(open(sys.argv[1]))
    shapes = {}
    for o in ops:
        if o["kind"] in ("conv", "convgn"):
            k = (o["M"], o["N"], o["K"])
            shapes.setdefault(k, [0, 0.0, o["H"]])
            shapes[k][0] += 1
            shapes[k][1] += o["ms"]
    tot_ours = tot_lib = 0.0
    print(f"{'M':>7} {'N':>5} {'K':>5} {'H':>3} {'n':>2} {'ours ms':>8} {'lib ms':>8} {'lib TF':>7}")
    for (M, N, K), (cnt, ms, H) in sorted(shapes.items(), key=lambda kv: -kv[1][1]):
        a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            torch.mm(a, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            torch.mm(a, b)
        e1.record()
        torch.cuda.synchronize()
        lib = e0.elapsed_time(e1) / reps
        tot_ours += ms
        tot_lib += lib * cnt
        print(f"{M:7d} {N:5d} {K:5d} {H:3d} {cnt:2d} {ms / cnt:8.4f} {lib:8.4f} {2 * M * N * K / lib / 1e9:7.1f}")
    print(f"total ours {tot_ours:.3f} ms, library GEMMs {tot_lib:.3f} ms")


if __name__ == "__main__":
    main()
