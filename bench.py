"""Benchmark: candidate-images/sec of the search-over-noise path (BASELINE.json metric).

One "step" = one RandomSearch round: N_local candidates per GPU x T=1000 DDPM steps
of the CIFAR-10 32x32 UNet (Arch A, config/config.yaml:25-29) in bf16 on MI355X,
the Oracle verifier on every candidate, one all_gather of the scores, argmax.
Weights: the seeded non-degenerate synthetic recipe (no checkpoint offline);
noise: Philox. Weak scaling: every GPU owns N_local candidates.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (driver, N > 1)

Rank 0 prints ONE JSON line. Extra fields: roofline (conv kernel census with HIP
events, same run) and cpu_baseline (the CPU oracle timed on this host's cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch
import torch.distributed as dist

MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md, chip-level table)
MFMA_FP32_PEAK_TFLOPS = 157.3


def cpu_baseline(T: int, seconds: float = 15.0, batch: int = 8):
    """Reference-equivalent CPU sampler (oracle, fp32) on this host's cores: UNet
    forwards of Arch A at batch `batch` for ~`seconds`, converted to candidate-images/s
    at T steps (img-fwd/s / T; the sampler update is negligible next to the forward)."""
    from oracle import ref_cpu as R
    from itsd.arch import ARCH_A
    from itsd.weights import synthetic_state_dict

    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)
    a = ARCH_A
    sd = synthetic_state_dict(a, 0)
    x = torch.randn(batch, 3, 32, 32)
    t = torch.full((batch,), 500, dtype=torch.long)
    sch = R.schedule(1e-4, 0.02, T)
    with torch.no_grad():
        fw = lambda xx, tt: R.unet_forward(sd, xx, tt, a.ch, a.ch_mult, a.attn, a.num_res_blocks)
        R.p_sample_loop(fw, x, sch, lambda s, xx: torch.randn_like(xx), t_begin=T - 1, t_end=T - 1, clip=False)
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            step = T - 1 - (n % (T - 1))
            x = R.p_sample_loop(fw, x, sch, lambda s, xx: torch.randn_like(xx), t_begin=step, t_end=step, clip=False)
            n += 1
        dt = time.perf_counter() - t0
    img_fwd_s = n * batch / dt
    return {"value": img_fwd_s / T, "unit": "candidate-images/sec", "cores": cores, "kind": "port",
            "sample": f"{n} sampler steps of Arch A fp32 at batch {batch} ({dt:.1f}s, {img_fwd_s:.2f} img-fwd/s), "
                      f"converted at T={T}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n-per-gpu", type=int, default=256)
    ap.add_argument("--T", type=int, default=1000)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import itsd
    from itsd.arch import ARCH_A, flops_per_image
    from itsd.diffusion import GaussianDiffusionSampler
    from itsd.model import UNet
    from itsd.search import SearchEngine
    from itsd.verifier import OracleVerifier

    a = ARCH_A
    n_local = args.n_per_gpu
    n_total = n_local * world
    net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=32, precision=args.precision,
               weights="gauss", seed=0, device=dev)
    smp = GaussianDiffusionSampler(net, 1e-4, 0.02, args.T)
    net.reserve(n_local)
    eng = SearchEngine(smp, OracleVerifier(), seed=1234, graph=not args.no_graph)
    shape = (1, 3, 32, 32)

    for w in range(args.warmup):
        eng.run_round(10_000 + w, n_total, shape)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    best = None
    for k in range(args.steps):
        r = eng.run_round(k, n_total, shape)
        best = (r.best_index, r.best_score)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())

    # Roofline of the dominant kernel: one census forward at the bench batch with HIP events
    # around every launch on the UNet's stream (itsd_profile_ops) picks the conv kind with the
    # most time ("convgnw" = conv3x3_gn_wide_kernel<1>, "convgnw4" = <4>, "convgn" =
    # conv3x3_gn_kernel, "conv" = the plain conv kernels); its launches are then timed in steady
    # state (itsd_profile_op). FLOPs are the MFMA work each launch executes.
    roof = None
    if rank == 0:
        x = torch.randn(n_local, 3, 32, 32, device=dev)
        t = torch.full((n_local,), 500, dtype=torch.int32, device=dev)
        nat = net.native(n_local)
        for _ in range(2):
            ops = nat.profile_ops(x, t)
        agg = {}
        for o in ops:
            if o["kind"] in ("conv", "convgn", "convgnw", "convgnw4"):
                g = agg.setdefault(o["kind"], [0, 0.0, 0.0])
                g[0] += 1
                g[1] += o["ms"]
                g[2] += o["flops"]
        kind = max(agg, key=lambda k: agg[k][1])
        n_l, ms_census, fl_sum = agg[kind]
        # per-launch time of the dominant kernel in steady state: each of its launches replayed
        # 10x back to back between HIP events on the UNet's stream (itsd_profile_op) -- what
        # the replayed step graph sees, without the eager census's per-launch event overhead
        ms_sum = sum(nat.profile_op(x, t, i, reps=10) for i, o in enumerate(ops) if o["kind"] == kind)
        avg_ms = ms_sum / n_l
        achieved = fl_sum / (ms_sum * 1e-3) / 1e12
        peak = MFMA_BF16_PEAK_TFLOPS if args.precision == "bf16" else MFMA_FP32_PEAK_TFLOPS
        total_ms = sum(o["ms"] for o in ops)
        conv_ms = sum(v[1] for v in agg.values())
        conv_fl = sum(v[2] for v in agg.values())
        names = {"convgn": "conv3x3_gn_kernel (fused GroupNorm+SiLU+conv3x3, 128x128 tile)",
                 "convgnw": "conv3x3_gn_wide_kernel<1> (fused GroupNorm+SiLU+conv3x3, 128x256 tile)",
                 "convgnw4": "conv3x3_gn_wide_kernel<4> (fused GroupNorm+SiLU+conv3x3, 8x8 level)",
                 "conv": "conv_pipe_wide / conv_pipe / conv_small (implicit-GEMM conv)"}
        traffic = None
        tfile = os.path.join(ROOT, "profiles", f"pmc_traffic_{kind}.json")
        if os.path.exists(tfile) and args.precision == "bf16" and n_local == 256:
            with open(tfile) as fh:
                traffic = json.load(fh).get("hbm_bytes_per_launch")
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "kernel": names[kind], "launches_per_forward": n_l, "avg_launch_ms": round(avg_ms, 4),
                "census_avg_launch_ms": round(ms_census / n_l, 4),
                "flops_per_launch": fl_sum / n_l,
                "traffic_source": os.path.relpath(tfile, ROOT) if traffic is not None else None,
                "all_conv_tflops": round(conv_fl / (conv_ms * 1e-3) / 1e12, 2),
                "conv_share_of_forward": round(conv_ms / total_ms, 4),
                "forward_ms": round(total_ms, 3),
                "forward_tflops_algorithmic": round(flops_per_image(a) * n_local / (total_ms * 1e-3) / 1e12, 2)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.T, seconds=args.cpu_seconds)

    if rank == 0:
        value = n_total * args.steps / dt
        out = {
            "metric": "candidate-images/sec at T=1000, CIFAR-10 32x32 UNet, N=256, 1/2/4/8 MI355X",
            "value": round(value, 3), "unit": "candidate-images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic (Philox noise, seeded non-degenerate random-init weights)",
            "config": {"workload": f"random-search round: N={n_local}/GPU candidates x T={args.T} DDPM steps, "
                                   f"Arch A UNet 32x32 (ch128 [1,2,3,4] attn[2] nrb2), Oracle verifier",
                       "model": "DDPM UNet (Diffusion/Model.py) Arch A", "global_batch": n_total, "seq_len": args.T,
                       "parallelism": f"candidate-dp{world}", "T": args.T, "graph": not args.no_graph,
                       "best_candidate": best},
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
