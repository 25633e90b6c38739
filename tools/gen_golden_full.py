"""Full-length golden trajectories from the REFERENCE ITSELF (build container only).

The reference's own samplers (``Diffusion/Diffusion.py:50-102``, ``DiffusionFreeGuidence/DiffusionCondition.py:
55-105``) are imported by file path from /root/reference (read-only, never copied) and their
``p_mean_variance`` is driven step by step over the WHOLE schedule with the throughput mode's Philox noise
(``oracle.ref_cpu.philox_normal``, bit-exact with the device generator: ``test_philox_noise_kernel_matches_oracle``),
replicating the loop body of ``forward`` (``x_t = mean + sqrt(var) * noise``, no noise at t = 0, NaN assert,
final clip). Each fixture holds only inputs and outputs -- the candidates' x_T, the denoised x0 and the
reference OracleVerifier's score (``search/verifier.py:45-66``), and x_0 before the final clip (the synthetic
model's full-length images saturate to +-1, so the clipped x0 alone would compare sign flips) -- for candidates of
the bench's shard rounds:

  full_C2  Arch A 32 px, T = 1000, a random-search round of N = 256 (engine seed 21), candidates 0 / 129 / 255
  full_C3  Arch C CFG (MainCondition.py), w = 1.8, betas 1e-4 .. 0.028, T = 1000, a zero-order round of the C3
           shard N_local = 32 (engine seed 41, round 1, pivot + 0.05 z, label 3), candidates 0 / 31
  full_C4  Arch A 64 px (example/imagenet_*.sh), T = 1000, a random round of the C4 shard N_local = 16 (seed 42),
           candidates 0 / 15
  full_C5  Arch A, T = 3000 (fine_tune_extended_T.py), a path-search round of the C5 shard N = 128 (seed 33,
           pivot + 0.1 z), candidates 0 / 64 / 127

The candidates' x_T and per-step noise follow itsd.search.SearchEngine (Philox of (seed, stream, global
element)): x_T = pivot + scale z in fp32 with one rounding (the device kernel's fused multiply-add), the
sampler's key (seed * 1000003 + round) mod 2^62. Weights: the seeded synthetic recipe (itsd.weights, seed 0).

    python tools/gen_golden_full.py [C2 C3 C4 C5]

The GPU box never runs this (it has no /root/reference); tests/test_gpu_full_T.py reads the fixtures.
"""
from __future__ import annotations

import contextlib
import dataclasses
import io
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_golden as G  # noqa: E402  (the reference loader and fixture writer)
from oracle import ref_cpu as R  # noqa: E402
from itsd.arch import ARCH_A, ARCH_C  # noqa: E402
from itsd.weights import synthetic_state_dict  # noqa: E402

STREAM_XT, STREAM_PERTURB, STREAM_INIT = 0xF0000000, 0xE0000000, 0xD0000000  # itsd.search


def philox(seed, stream, lo, n, shape):
    return R.philox_normal(seed, stream, np.arange(lo, lo + n)).reshape(shape)


def fma_f32(scale: float, z: torch.Tensor, pivot: torch.Tensor) -> torch.Tensor:
    """fp32 pivot + scale z with one rounding (the product of two fp32 values is exact in fp64)."""
    s = np.float64(np.float32(scale))
    return (s * z.double() + pivot.double()).float()


def candidates(kind, seed, round_id, cands, per, shape, scale=1.0):
    if kind == "random":
        return torch.stack([philox(seed, STREAM_XT + round_id, i * per, per, shape) for i in cands]), None
    pivot = philox(seed, STREAM_INIT, 0, per, shape)
    xs = [fma_f32(scale, philox(seed, STREAM_PERTURB + round_id, i * per, per, shape), pivot) for i in cands]
    return torch.stack(xs), pivot


def drive(sampler, x_T, run_seed, cands, per, T, labels=None):
    """``forward``'s loop (Diffusion.py:88-102 / DiffusionCondition.py:92-105) with Philox noise per step."""
    x_t = x_T.clone()
    shape = tuple(x_T.shape[1:])
    t0 = time.time()
    with torch.no_grad():
        for time_step in reversed(range(T)):
            t = x_t.new_ones([x_T.shape[0], ], dtype=torch.long) * time_step
            if labels is None:
                mean, var = sampler.p_mean_variance(x_t=x_t, t=t)
            else:
                mean, var = sampler.p_mean_variance(x_t=x_t, t=t, labels=labels)
            if time_step > 0:
                noise = torch.stack([philox(run_seed, time_step, i * per, per, shape) for i in cands])
            else:
                noise = 0
            x_t = mean + torch.sqrt(var) * noise
            assert torch.isnan(x_t).int().sum() == 0, "nan in tensor."
            if time_step % 200 == 0:
                print(f"    t={time_step} ({time.time() - t0:.0f}s)", flush=True)
    return torch.clip(x_t, -1, 1), x_t  # (the reference's return value; and x_0 before its clip)


def main():
    only = sys.argv[1:] or ["C2", "C3", "C4", "C5"]
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    M = G._load("ref_model", "Diffusion/Model.py")
    D = G._load("ref_diffusion", "Diffusion/Diffusion.py")
    MC = G._load("ref_model_cond", "DiffusionFreeGuidence/ModelCondition.py")
    DC = G._load("ref_diffusion_cond", "DiffusionFreeGuidence/DiffusionCondition.py")
    G._stub_torchvision()
    with contextlib.redirect_stdout(io.StringIO()):
        V = G._load("ref_verifier", "search/verifier.py")
    ov = V.OracleVerifier()
    score = lambda x0: np.array([np.float64(ov.score(x0[i:i + 1])) for i in range(x0.shape[0])])
    run_key = lambda seed, rnd: (seed * 1000003 + rnd) & ((1 << 62) - 1)  # SearchEngine.run_round

    def ddpm(a, T, bT):
        return D.GaussianDiffusionSampler(G.ref_ddpm(M, a, synthetic_state_dict(a, 0)), 1e-4, bT, T)

    with torch.no_grad():
        if "C2" in only:
            a, T, seed, rnd, cands = ARCH_A, 1000, 21, 0, (0, 129, 255)
            per, shape = 3 * 32 * 32, (3, 32, 32)
            x_T, _ = candidates("random", seed, rnd, cands, per, shape)
            print("full_C2", flush=True)
            x0, raw = drive(ddpm(a, T, 0.02), x_T, run_key(seed, rnd), cands, per, T)
            G.save("full_C2", seed=seed, round=rnd, n=256, cands=np.array(cands), T=T, beta_T=0.02, x_T=x_T, x0=x0,
                   x0_raw=raw, scores=score(x0))
        if "C3" in only:
            a, T, seed, rnd, cands, w, lab = ARCH_C, 1000, 41, 1, (0, 31), 1.8, 3
            per, shape = 3 * 32 * 32, (3, 32, 32)
            x_T, pivot = candidates("zero_order", seed, rnd, cands, per, shape, scale=1 - 0.95)
            net = G.ref_cfg(MC, a, synthetic_state_dict(a, 0))
            smp = DC.GaussianDiffusionSampler(net, 1e-4, 0.028, T, w=w)
            print("full_C3", flush=True)
            x0, raw = drive(smp, x_T, run_key(seed, rnd), cands, per, T, labels=torch.full((len(cands),), lab))
            G.save("full_C3", seed=seed, round=rnd, n=32, cands=np.array(cands), T=T, beta_T=0.028, w=w, label=lab,
                   scale=np.float32(1 - 0.95), x_T=x_T, pivot=pivot, x0=x0, x0_raw=raw, scores=score(x0))
        if "C4" in only:
            a, T, seed, rnd, cands = dataclasses.replace(ARCH_A, img_size=64), 1000, 42, 0, (0, 15)
            per, shape = 3 * 64 * 64, (3, 64, 64)
            x_T, _ = candidates("random", seed, rnd, cands, per, shape)
            print("full_C4", flush=True)
            x0, raw = drive(ddpm(a, T, 0.02), x_T, run_key(seed, rnd), cands, per, T)
            G.save("full_C4", seed=seed, round=rnd, n=16, cands=np.array(cands), T=T, beta_T=0.02, x_T=x_T, x0=x0,
                   x0_raw=raw, scores=score(x0))
        if "C5" in only:
            a, T, seed, rnd, cands = dataclasses.replace(ARCH_A, T=3000), 3000, 33, 0, (0, 64, 127)
            per, shape = 3 * 32 * 32, (3, 32, 32)
            x_T, pivot = candidates("path", seed, rnd, cands, per, shape, scale=0.1)
            print("full_C5", flush=True)
            x0, raw = drive(ddpm(a, T, 0.02), x_T, run_key(seed, rnd), cands, per, T)
            G.save("full_C5", seed=seed, round=rnd, n=128, cands=np.array(cands), T=T, beta_T=0.02,
                   scale=np.float32(0.1), x_T=x_T, pivot=pivot, x0=x0, x0_raw=raw, scores=score(x0))
    print("torch", torch.__version__)


if __name__ == "__main__":
    main()
