"""Benchmark: candidate-images/sec of the search-over-noise path (BASELINE.json metric).

One "step" = one RandomSearch round: N_local candidates per GPU x T=1000 DDPM steps
of the CIFAR-10 32x32 UNet (Arch A, config/config.yaml:25-29) in bf16 on MI355X,
the Oracle verifier on every candidate, one all_gather of the scores, argmax.
Weights: the seeded non-degenerate synthetic recipe (no checkpoint offline);
noise: Philox. The metric's N = 256 candidates per round are split over the GPUs (strong
scaling, N_local = 256 / n_gpus); --n-per-gpu N runs N per GPU instead (weak scaling), and a
multi-GPU run also reports the N = 256-per-GPU weak-scaling rate as a side field.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n N | --n-per-gpu N] [--no-extras]
    torchrun --nproc-per-node N bench.py --gpus N ...      (driver, N > 1)

Rank 0 prints ONE JSON line. Extra fields (single-GPU runs):
  roofline      the dominant kernel (fused GroupNorm conv) in steady state with HIP events on
                the UNet's stream, its PMC HBM traffic (profiles/, this commit), the conv tiles'
                HBM GB/s, and the attention kernels' MFMA utilisation;
  sweep         N in {8, 16, 32, 64, 128, 256, 1024} on one GPU (north_star's N set; N = 32 / 64 / 128 are
                the 8- / 4- / 2-GPU shards of N = 256, N = 8 / 16 those of N = 64 at 8 / 4 GPUs), same path;
  fp32          the reference-precision (parity mode) throughput at the headline N, a full T-step round;
  legs          the other BASELINE configs per GPU shard: C3 CFG zero-order round (Arch C,
                N_local = 32 -> 2N = 64 guided batch), C4 64x64 Arch A (N_local = 16), C5
                T = 3000 path search (N_local = 128), each with its own dominant kernel;
  cpu_baseline  the CPU oracle (fp32) timed on this host's cores at B in {1, 8, 32} plus a
                full-loop conversion check (equal interleaved windows, `agrees` within 15 %).
Windowed lines time a contiguous window of sampler steps (every DDPM step runs the same
UNet, so candidate-images/s at T = N / (T x per-step time)); the window is stated in each.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch
import torch.distributed as dist

MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md, chip-level table)
MFMA_FP32_PEAK_TFLOPS = 157.3
HBM_PEAK_GBPS = 8000.0
CONV_KINDS = ("conv", "convgn", "convgnw", "convgnw4")
KERNEL_NAMES = {  # op classes of the census
    "convgn": "fused GroupNorm+SiLU+conv3x3, 128-pixel tiles",
    "convgnw": "fused GroupNorm+SiLU+conv3x3, 256-pixel tiles (32x32 / 16x16 levels)",
    "convgnw4": "fused GroupNorm+SiLU+conv3x3, 256-pixel tiles of four 8x8 images",
    "conv": "implicit-GEMM conv (1x1, strided, sub-pixel upsample, 4x4 level)",
    "attn": "self-attention on MFMA",
    "attnblock": "fused AttnBlock (GroupNorm + q|k|v + attention + proj)",
}


def cpu_baseline(T: int, seconds: float = 12.0, check_seconds: float = 10.0):
    """Reference-equivalent CPU sampler (oracle, fp32) on this host's cores: UNet forwards of
    Arch A at B in {1, 8, 32} (seconds/3 each), converted to candidate-images/s at T
    (img-fwd/s / T; the sampler update is negligible next to the forward).

    Conversion check: the full N = 1 ancestral loop (R.p_sample_loop, short T) and B = 1
    forwards, each timed over an equal window of check_seconds, interleaved twice (loop,
    forwards, loop, forwards) so that host-frequency drift or a neighbour's load hits both
    legs alike; the best of each is compared and `agrees` is true within +-15 %."""
    from oracle import ref_cpu as R
    from itsd.arch import ARCH_A
    from itsd.weights import synthetic_state_dict

    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)  # once, before any CPU op (the intra-op pool is sized here)
    a = ARCH_A
    sd = synthetic_state_dict(a, 0)
    fw = lambda xx, tt: R.unet_forward(sd, xx, tt, a.ch, a.ch_mult, a.attn, a.num_res_blocks)

    def fwd_rate(b, window):
        x = torch.randn(b, 3, 32, 32)
        t = torch.full((b,), 500, dtype=torch.long)
        fw(x, t)  # untimed: this batch's allocations (the caching allocator keeps them) and kernel choices
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < window or n == 0:
            fw(x, t)
            n += 1
        return n * b / (time.perf_counter() - t0)

    def loop_rate(window):
        Tc = 10
        sc = R.schedule(1e-4, 0.02, Tc)
        steps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < window or steps == 0:
            R.p_sample_loop(fw, torch.randn(1, 3, 32, 32), sc, lambda s, xx: torch.randn_like(xx))
            steps += Tc
        return steps / (time.perf_counter() - t0)

    per_b = {}
    with torch.no_grad():
        fwd_rate(1, 0.5)  # warm the thread pool and the allocator
        for b in (1, 8, 32):
            per_b[b] = fwd_rate(b, seconds / 3)
        loops, fwds = [], []
        for _ in range(2):
            loops.append(loop_rate(check_seconds / 2))
            fwds.append(fwd_rate(1, check_seconds / 2))
    best_b = max(per_b, key=per_b.get)
    lr, fr = max(loops), max(fwds)
    dev = (lr - fr) / fr
    return {"value": per_b[best_b] / T, "unit": "candidate-images/sec", "cores": cores, "kind": "port",
            "sample": f"Arch A fp32 UNet forwards at B=1/8/32: {per_b[1]:.2f}/{per_b[8]:.2f}/{per_b[32]:.2f} "
                      f"img-fwd/s ({seconds / 3:.0f}s each), value = best (B={best_b}) / T={T}; "
                      f"check: full N=1 loop {lr:.2f} steps/s vs B=1 forwards {fr:.2f} img-fwd/s "
                      f"({check_seconds:.0f}s each, interleaved)",
            "img_fwd_per_s": {str(k): round(v, 3) for k, v in per_b.items()},
            "full_loop_check": {"N": 1, "window_s": check_seconds, "loop_steps_per_s": [round(v, 3) for v in loops],
                                "b1_fwd_per_s": [round(v, 3) for v in fwds], "deviation": round(dev, 4),
                                "agrees": abs(dev) <= 0.15}}


def census(net, n: int, img: int, labels=None):
    """Per-launch census of one forward (HIP events on the UNet's stream): per kind
    [launches, ms, flops] and the op list."""
    dev = net.device
    x = torch.randn(n, 3, img, img, device=dev)
    t = torch.full((n,), 500, dtype=torch.int32, device=dev)
    nat = net.native(n)
    for _ in range(2):
        ops = nat.profile_ops(x, t)
    agg = {}
    for o in ops:
        g = agg.setdefault(o["kind"], [0, 0.0, 0.0])
        g[0] += 1
        g[1] += o["ms"]
        g[2] += o["flops"]
    return ops, agg, nat, x, t


def conv_alg_bytes(o) -> float:
    """Algorithmic HBM bytes of one bf16 conv launch, every operand once: input activations, weights,
    output, the residual operand when the op adds one (ResBlock block2 / shortcut sums, Model.py:184),
    the output's GroupNorm statistics slab (fp32 sum and square sum per channel and slot of
    min(HW, 128) pixels), for a fused GroupNorm+SiLU input the input's statistics slab read, and for a
    folded 1x1 shortcut (K slices of the block2 conv) the shortcut's input and weights."""
    ks = max(1, o["ks"])
    cin = o["K"] // (ks * ks)
    su = o["stride_up"]
    stride, ups = su // 10, su % 10
    m_in = o["M"] * stride * stride if not ups else o["M"] // 4
    b = 2.0 * (m_in * cin + o["N"] * o["K"] + o["M"] * o["N"])
    if o.get("resid"):
        b += 2.0 * o["M"] * o["N"]
    hw_out = o["H"] * o["H"]
    if o.get("stats_out"):
        b += 4.0 * 2 * (o["M"] / min(hw_out, 128)) * o["N"]
    if o.get("gn_in"):
        hw_in = hw_out * stride * stride if not ups else hw_out // 4
        b += 4.0 * 2 * (m_in / min(hw_in, 128)) * cin
    if o.get("sc_cin"):  # a ResBlock 1x1 shortcut folded in as K slices: its input and weights (no residual operand)
        b += 2.0 * (o["M"] * o["sc_cin"] + o["N"] * o["sc_cin"])
    return b


def rocprof_name(kernel: str) -> str:
    """The census kernel name (the ITSD_LAUNCH expression) as rocprofv3 prints it (bf16 builds)."""
    k = kernel.strip("()").replace("<T,", "<unsigned short,").replace("<T>", "<unsigned short>")
    return k


def kernel_file(kernel: str) -> str:
    return "".join(ch if ch.isalnum() else "_" for ch in rocprof_name(kernel)).strip("_")


def kernel_function(kernel: str) -> str:
    """The kernel FUNCTION of a census kernel name: template arguments dropped
    ("conv3x3_gn_p4_kernel<32>" -> "conv3x3_gn_p4_kernel")."""
    return rocprof_name(kernel).split("<")[0]


def live_traffic(kernels, n: int, timeout_s: float = 150.0):
    """HBM bytes per launch of each kernel instantiation, measured in THIS run: two rocprofv3
    --pmc passes (FETCH_SIZE, then WRITE_SIZE: separate runs, no tracing domains) over one census
    forward in a child process, reduced by tools/pmc_traffic.py (FETCH_SIZE x 2 on gfx950 +
    WRITE_SIZE). Returns {kernel: bytes} or None when the profiler is unavailable or fails."""
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    env = dict(os.environ, TMPDIR="/tmp")
    d = tempfile.mkdtemp(prefix="itsd_pmc_", dir="/tmp")
    try:
        for i, ctr in enumerate(("FETCH_SIZE", "WRITE_SIZE")):
            cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", os.path.join(d, f"p{i}"), "-o", "run", "--",
                   sys.executable, os.path.join(ROOT, "tools", "census.py"), "--reps", "1", "--n", str(n)]
            r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout_s)
            if r.returncode != 0:
                return None
        out = {}
        for k in kernels:
            js = os.path.join(d, "t.json")
            r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), d, k, js], cwd=ROOT,
                               capture_output=True, text=True, timeout=60)
            if r.returncode != 0 or not os.path.exists(js):
                return None
            with open(js) as fh:
                out[k] = json.load(fh)["hbm_bytes_per_launch"]
            os.remove(js)
        return out
    except Exception:
        return None
    finally:
        shutil.rmtree(d, ignore_errors=True)


def dominant_roofline(ops, agg, nat, x, t, precision: str, steady: bool = True):
    """Roofline of the conv kernel FUNCTION (all its template instantiations, e.g. the fused
    conv at 32x32 / 16x16 / 8x8) with the most time in the census forward; the per-instantiation
    launch counts and times are listed beside it for the rocprof cross-check."""
    per = {}
    for i, o in enumerate(ops):
        if o["kind"] in CONV_KINDS:
            name = o["kernel"] or o["kind"]
            g = per.setdefault(kernel_function(name), [0, 0.0, 0.0, [], o["kind"], {}])
            g[0] += 1
            g[1] += o["ms"]
            g[2] += o["flops"]
            g[3].append(i)
            g[5].setdefault(name, []).append(i)
    func = max(per, key=lambda k: per[k][1])
    n_l, ms_census, fl_sum, idx, kind, inst = per[func]
    # each launch replayed 10x back to back between HIP events (itsd_profile_op): what the
    # replayed step graph sees, without the eager census's per-launch event overhead
    ms_of = {i: (nat.profile_op(x, t, ops[i]["op"], reps=10) if steady else ops[i]["ms"]) for i in idx}
    ms_sum = sum(ms_of.values())
    achieved = fl_sum / (ms_sum * 1e-3) / 1e12
    peak = MFMA_BF16_PEAK_TFLOPS if precision == "bf16" else MFMA_FP32_PEAK_TFLOPS
    insts = []
    for name, ii in sorted(inst.items(), key=lambda kv: -sum(ms_of[i] for i in kv[1])):
        ims = sum(ms_of[i] for i in ii)
        ifl = sum(ops[i]["flops"] for i in ii)
        insts.append({"kernel": rocprof_name(name), "launches_per_forward": len(ii),
                      "avg_launch_ms": round(ims / len(ii), 4), "tflops": round(ifl / (ims * 1e-3) / 1e12, 2),
                      "alg_bytes": round(sum(conv_alg_bytes(ops[i]) for i in ii) / len(ii))})
    return func, {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                  "frac": round(achieved / peak, 4), "kernel": func,
                  "family": KERNEL_NAMES[kind], "launches_per_forward": n_l,
                  "avg_launch_ms": round(ms_sum / n_l, 4), "census_avg_launch_ms": round(ms_census / n_l, 4),
                  "flops_per_launch": fl_sum / n_l, "instantiations": insts}


def windowed_rate(smp, n: int, img: int, T: int, window: int, labels=None, rounds: int = 1):
    """Candidate-images/s at T from a timed window of `window` sampler steps (t = T-1 ..)."""
    dev = smp.model.device
    x = torch.randn(n, 3, img, img, device=dev)
    lab = labels
    warm = min(window, 50)  # (the step graph is captured on the first step; a full-length window needs no full warm run)
    smp.run(x, t_begin=T - 1, t_end=T - warm, labels=lab, seed=7, clip=False)  # capture + warm
    torch.cuda.synchronize()
    best = None
    for _ in range(rounds):
        x = torch.randn(n, 3, img, img, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        smp.run(x, t_begin=T - 1, t_end=T - window, labels=lab, seed=11, clip=False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    ms_step = best / window * 1e3
    return n / (T * ms_step * 1e-3), ms_step


def progress(msg: str) -> None:
    """A progress line on stderr (long runs must show life within minutes; stdout is the JSON)."""
    print(f"[bench] {time.strftime('%H:%M:%S')} {msg}", file=sys.stderr, flush=True)


def leg(name, make_net, n: int, img: int, T: int, window: int, cfg: bool, precision: str = "bf16",
        workload: str = ""):
    from itsd.diffusion import CondGaussianDiffusionSampler, GaussianDiffusionSampler

    progress(f"leg {name}: {workload}")
    net = make_net()
    net.reserve(2 * n if cfg else n)
    if cfg:
        smp = CondGaussianDiffusionSampler(net, 1e-4, 0.028, T, w=1.8)
        labels = (torch.arange(n, device=net.device) % 10 + 1).to(torch.int32)
    else:
        smp = GaussianDiffusionSampler(net, 1e-4, 0.02, T)
        labels = None
    rate, ms_step = windowed_rate(smp, n, img, T, window, labels)
    out = {"workload": workload, "value": round(rate, 4), "unit": "candidate-images/sec per GPU",
           "ms_per_step": round(ms_step, 3), "T": T, "N_local": n, "dtype": precision,
           "sample": f"steps t={T - 1}..{T - window} ({window} of {T}) timed, converted to T={T}"}
    try:
        bn = 2 * n if cfg else n
        ops, agg, nat, x, t = census(net, bn, img)
        _, roof = dominant_roofline(ops, agg, nat, x, t, precision)
        out["roofline"] = roof
    except Exception as e:  # the leg's number stands without its census
        out["roofline_error"] = repr(e)
    del smp, net
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", "--n-total", dest="n_total", type=int, default=256,
                    help="global N of the metric (N=256), split over the GPUs: strong scaling (default)")
    ap.add_argument("--n-per-gpu", type=int, default=0, help="weak scaling instead: N per GPU")
    ap.add_argument("--T", type=int, default=1000)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip sweep / fp32 / legs")
    ap.add_argument("--no-live-traffic", action="store_true",
                    help="take the dominant kernel's HBM traffic from profiles/ instead of two PMC passes")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-weak-line", action="store_true", help="(N > 1) skip the N=256-per-GPU weak-scaling field")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # under torchrun (any world size, 1 included) the ranks form an RCCL group and the round
    # protocol runs its collectives; a plain `python bench.py` runs without one
    use_pg = "WORLD_SIZE" in os.environ and "MASTER_ADDR" in os.environ
    if use_pg:
        dist.init_process_group("nccl", device_id=dev)

    import itsd
    from itsd.arch import ARCH_A, ARCH_C, flops_per_image
    from itsd.diffusion import GaussianDiffusionSampler
    from itsd.model import CondUNet, UNet
    from itsd.search import SearchEngine
    from itsd.verifier import OracleVerifier

    a = ARCH_A
    if args.n_per_gpu:
        n_local, scaling = args.n_per_gpu, "weak"
        n_total = n_local * world
    else:  # the metric's N = 256 candidates per round, split over the GPUs
        if args.n_total % world:
            raise SystemExit(f"--n {args.n_total} does not split over {world} GPUs")
        n_total, n_local, scaling = args.n_total, args.n_total // world, "strong"
    net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=32, precision=args.precision,
               weights="gauss", seed=0, device=dev)
    smp = GaussianDiffusionSampler(net, 1e-4, 0.02, args.T)
    net.reserve(n_local)
    eng = SearchEngine(smp, OracleVerifier(), seed=1234, graph=not args.no_graph)
    shape = (1, 3, 32, 32)

    if rank == 0:
        progress(f"warmup x{args.warmup}, then {args.steps} timed rounds of N={n_total}")
    for w in range(args.warmup):
        eng.run_round(10_000 + w, n_total, shape)
    torch.cuda.synchronize()
    if use_pg:
        dist.barrier()
    t0 = time.perf_counter()
    best = None
    for k in range(args.steps):
        r = eng.run_round(k, n_total, shape)
        best = (r.best_index, r.best_score)
    torch.cuda.synchronize()
    if use_pg:
        dist.barrier()
    dt = time.perf_counter() - t0
    if use_pg:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())

    # N > 1 with the metric's fixed N = 256: also the weak-scaling rate (N = 256 per GPU, the same
    # round protocol over the same ranks) as a side field; the headline stays the metric's N
    weak = None
    if world > 1 and scaling == "strong" and not args.no_weak_line:
        nw = 256 * world
        net.reserve(256)
        eng.run_round(20_000, nw, shape)  # capture the N_local = 256 graph
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for k in range(args.steps):
            eng.run_round(30_000 + k, nw, shape)
        torch.cuda.synchronize()
        dist.barrier()
        tw = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
        dist.all_reduce(tw, op=dist.ReduceOp.MAX)
        weak = {"value": round(nw * args.steps / float(tw.item()), 3), "unit": "candidate-images/sec",
                "global_batch": nw, "n_local": 256, "steps": args.steps, "scaling": "weak",
                "ms_per_step": round(float(tw.item()) / args.steps * 1e3, 2)}

    roof = None
    if rank == 0:
        progress(f"headline: {n_total * args.steps / dt:.3f} candidate-images/s; roofline census")
        ops, agg, nat, x, t = census(net, n_local, 32)
        kernel, roof = dominant_roofline(ops, agg, nat, x, t, args.precision)
        n_l = roof["launches_per_forward"]
        total_ms = sum(o["ms"] for o in ops)
        conv_ms = sum(v[1] for k, v in agg.items() if k in CONV_KINDS)
        conv_fl = sum(v[2] for k, v in agg.items() if k in CONV_KINDS)
        # HBM traffic of the dominant kernel: PMC passes of this commit (tools/pmc_passes.sh at
        # N = 256, corrected as MI355X_MICROARCH.md prescribes), per launch
        # (launch-weighted over the function's instantiations): measured live in this run by two
        # PMC passes of a child process; else (profiler unavailable) from this commit's committed
        # PMC files at N = 256; null unless every instantiation has a number
        traffic, tfiles = None, []
        live = None
        if args.precision == "bf16" and not args.no_live_traffic and world == 1:
            progress("PMC traffic passes (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, child process)")
            live = live_traffic([ins["kernel"] for ins in roof["instantiations"]], n_local)
        if live is not None:
            tot_b = sum(live[ins["kernel"]] * ins["launches_per_forward"] for ins in roof["instantiations"])
            tot_n = sum(ins["launches_per_forward"] for ins in roof["instantiations"])
            for ins in roof["instantiations"]:
                ins["traffic"] = live[ins["kernel"]]
                ins["traffic_ratio"] = round(ins["traffic"] / ins["alg_bytes"], 3)  # PMC / algorithmic bytes
            traffic = tot_b / tot_n
            tfiles = "live: rocprofv3 --pmc FETCH_SIZE (x2) + WRITE_SIZE in this run"
        elif args.precision == "bf16" and n_local == 256:
            tot_b, tot_n = 0.0, 0
            for ins in roof["instantiations"]:
                tfile = os.path.join(ROOT, "profiles", f"pmc_traffic_{kernel_file(ins['kernel'])}.json")
                if not os.path.exists(tfile):
                    tot_n = -1
                    break
                with open(tfile) as fh:
                    tb = json.load(fh).get("hbm_bytes_per_launch")
                ins["traffic"] = tb
                ins["traffic_ratio"] = round(tb / ins["alg_bytes"], 3)
                tot_b += tb * ins["launches_per_forward"]
                tot_n += ins["launches_per_forward"]
                tfiles.append(os.path.relpath(tfile, ROOT))
            if tot_n > 0:
                traffic = tot_b / tot_n
        dom = [o for o in ops if o["kind"] in CONV_KINDS and kernel_function(o["kernel"] or o["kind"]) == kernel]
        alg_b = sum(conv_alg_bytes(o) for o in dom) / len(dom)
        avg_s = roof["avg_launch_ms"] * 1e-3
        # on-box calibration ("re-measure both on the box"): the achievable bf16 MFMA rate
        # (random operands, every CU) and HBM streaming rate of THIS device, and the fractions against
        # them, so that a round-to-round delta can be told from the +-5-8 % spread between boxes
        calib = None
        try:
            from itsd import runtime as rt
            progress("calibration: bf16 MFMA loop, HBM copy")
            mf, hb = rt.calibrate(rt.CALIB_MFMA_BF16), rt.calibrate(rt.CALIB_HBM_COPY)
            mf16 = rt.calibrate(rt.CALIB_MFMA_BF16_16X16)
            calib = {"mfma_bf16_tflops": round(mf, 1), "mfma_bf16_16x16x32_tflops": round(mf16, 1),
                     "hbm_copy_gbps": round(hb, 1),
                     "mfma_frac_of_spec": round(mf / MFMA_BF16_PEAK_TFLOPS, 4),
                     "hbm_frac_of_spec": round(hb / HBM_PEAK_GBPS, 4),
                     "method": "v_mfma_f32_32x32x16_bf16 chains (the fused convs' shape; 16x16x32 beside it) on "
                               "random operands, 2 waves/SIMD on every CU; "
                               "1 GiB 16-B/lane copy (read + write bytes); best of 3 after a warm launch"}
            if args.precision == "bf16":
                calib["dominant_frac_of_measured"] = round(roof["achieved"] / mf, 4)
        except Exception as e:  # the line stands without it
            calib = {"error": repr(e)}
        roof["calibration"] = calib
        roof.update({
            "traffic": traffic,
            "traffic_source": tfiles if traffic is not None else None,
            "all_conv_tflops": round(conv_fl / (conv_ms * 1e-3) / 1e12, 2),
            "conv_share_of_forward": round(conv_ms / total_ms, 4),
            "forward_ms": round(total_ms, 3),
            "forward_tflops_algorithmic": round(flops_per_image(a) * n_local / (total_ms * 1e-3) / 1e12, 2),
            # north_star: HBM GB/s of the conv tiles (dominant kernel) against the 8 TB/s peak
            "conv_hbm": {"kernel": kernel, "alg_bytes_per_launch": alg_b,
                         "alg_gbps": round(alg_b / avg_s / 1e9, 1),
                         "pmc_bytes_per_launch": traffic,
                         "pmc_gbps": round(traffic / avg_s / 1e9, 1) if traffic else None,
                         "pmc_frac_of_peak": round(traffic / avg_s / 1e9 / HBM_PEAK_GBPS, 4) if traffic else None,
                         "pmc_frac_of_measured": (round(traffic / avg_s / 1e9 / calib["hbm_copy_gbps"], 4)
                                                  if traffic and calib and calib.get("hbm_copy_gbps") else None),
                         "traffic_ratio": round(traffic / alg_b, 3) if traffic else None,
                         "peak_gbps": HBM_PEAK_GBPS},
        })
        # attention (north_star: MFMA utilisation): the fused AttnBlock kernel (GroupNorm, q|k|v and
        # proj projections, softmax attention in one launch; its FLOPs are all of those) and the
        # plain attention kernel where an AttnBlock is not fused (the 4x4 level)
        att = {}
        for kind in ("attnblock", "attn"):
            if kind in agg:
                al, ams, afl = agg[kind]
                at = afl / (ams * 1e-3) / 1e12
                akern = sorted({rocprof_name(o["kernel"]) for o in ops if o["kind"] == kind})
                att[kind] = {"kernel": " / ".join(akern), "launches_per_forward": al,
                             "avg_launch_ms": round(ams / al, 4), "tflops": round(at, 2),
                             "mfma_frac": round(at / MFMA_BF16_PEAK_TFLOPS, 4),
                             "share_of_forward": round(ams / total_ms, 4)}
        if att:
            roof["attention"] = att.get("attnblock", att.get("attn"))
            if len(att) > 1:
                roof["attention"]["unfused"] = att["attn"]

    extras = {}
    if rank == 0 and world == 1 and not args.no_extras:
        # north_star N sweep on the same path (headline N is the main line)
        sweep = {}
        for n, window in ((8, 1000), (16, 1000), (32, 1000), (64, 1000), (128, 1000), (256, 1000), (1024, 100)):
            if n == n_local:
                continue
            progress(f"sweep N={n}")
            net.reserve(n)
            rate, ms = windowed_rate(smp, n, 32, args.T, window)
            sweep[str(n)] = {"value": round(rate, 3), "ms_per_step": round(ms, 3),
                             "sample": f"{window} of {args.T} steps timed"}
        sweep[str(n_local)] = {"value": round(n_total * args.steps / dt, 3), "ms_per_step":
                               round(dt / args.steps / args.T * 1e3, 3), "sample": "headline"}
        extras["sweep"] = {"unit": "candidate-images/sec", "T": args.T, "dtype": args.precision, "points": sweep}
        del eng, smp, net, nat
        torch.cuda.empty_cache()
        if args.precision == "bf16":
            extras["fp32"] = leg("fp32", lambda: UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0,
                                                      img_size=32, precision="fp32", weights="gauss", seed=0,
                                                      device=dev),
                                 n_local, 32, args.T, args.T, cfg=False, precision="fp32",
                                 workload=f"Arch A 32 px, N={n_local}, fp32 parity mode (the reference's precision)")
        c = ARCH_C
        extras["legs"] = {
            "C3": leg("C3", lambda: CondUNet(c.T, c.num_labels, c.ch, c.ch_mult, c.num_res_blocks, 0.0, img_size=32,
                                             precision="bf16", weights="gauss", seed=0, device=dev),
                      32, 32, 1000, 50, cfg=True,
                      workload="CFG zero-order round per GPU shard: Arch C (MainCondition.py), N_local=32 "
                               "(2N=64 guided batch), T=1000, w=1.8"),
            "C4": leg("C4", lambda: UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=64,
                                         precision="bf16", weights="gauss", seed=0, device=dev),
                      16, 64, 1000, 50, cfg=False,
                      workload="64x64 Arch A per GPU shard (N=128 over 8 GPUs): N_local=16, T=1000"),
            "C5": leg("C5", lambda: UNet(3000, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=32,
                                         precision="bf16", weights="gauss", seed=0, device=dev),
                      128, 32, 3000, 100, cfg=False,
                      workload="T=3000 path search per GPU shard (N=1024 over 8 GPUs): N_local=128, "
                               "fine_tune_extended_T.py schedule"),
        }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("cpu baseline")
        cpu = cpu_baseline(args.T, seconds=args.cpu_seconds)

    if rank == 0:
        value = n_total * args.steps / dt
        out = {
            "metric": "candidate-images/sec at T=1000, CIFAR-10 32x32 UNet, N=256, 1/2/4/8 MI355X",
            "value": round(value, 3), "unit": "candidate-images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic (Philox noise, seeded non-degenerate random-init weights)",
            "config": {"workload": f"random-search round: N={n_local}/GPU candidates x T={args.T} DDPM steps, "
                                   f"Arch A UNet 32x32 (ch128 [1,2,3,4] attn[2] nrb2), Oracle verifier",
                       "model": "DDPM UNet (Diffusion/Model.py) Arch A", "global_batch": n_total, "seq_len": args.T,
                       "parallelism": f"candidate-dp{world}", "T": args.T, "graph": not args.no_graph,
                       "process_group": dist.get_backend() if use_pg else None, "n_local": n_local,
                       "best_candidate": best},
            "roofline": roof, "cpu_baseline": cpu,
        }
        if weak is not None:
            out["weak_scaling"] = weak
        out.update(extras)
        print(json.dumps(out), flush=True)
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
