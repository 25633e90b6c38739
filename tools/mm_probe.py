"""Library GEMM (torch.mm -> hipBLASLt) time for the 1x1-conv shapes of the N=256 forward, against
the HBM floor of the same bytes (measurement only, never part of the product).

    python tools/mm_probe.py
"""
import torch

SHAPES = [(262144, 384, 128), (262144, 256, 128), (65536, 640, 256), (65536, 512, 256), (65536, 384, 256),
          (16384, 896, 384), (16384, 768, 384), (16384, 640, 384), (4096, 1024, 512)]


def main():
    for M, K, N in SHAPES:
        a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            torch.mm(a, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 50
        e0.record()
        for _ in range(reps):
            torch.mm(a, b)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        byts = (M * K + K * N + M * N) * 2
        print(f"M={M:7d} K={K:5d} N={N:4d}: {ms * 1e3:7.1f} us  {byts / ms / 1e9:6.0f} GB/s  "
              f"HBM floor {byts / 8e12 * 1e6:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
