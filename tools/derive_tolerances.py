"""Derive the full-length parity tolerances of tests/test_gpu_full_T.py from measured drift (VERDICT r4 #5c).
Test infrastructure (runs the CPU oracle only); writes tests/golden/tolerance_derivation.json.

Two measurements, each a whole ancestral loop (Diffusion/Diffusion.py:84-102; CFG DiffusionCondition.py:89-105)
of the oracle on CPU, on the same x_T and Philox noise as the GPU tests:

  fp32 drift   the fp32 oracle against the SAME loop in fp64 (weights, activations and x in float64; the
               schedule coefficients are the reference's fp32 casts in both, Diffusion.py:9-16). The GPU fp32
               path (exact-product f32 MFMA, other summation orders) and the fp32 oracle are two fp32
               evaluations of one fp64 trajectory: |GPU - oracle| <= |GPU - fp64| + |oracle - fp64|, and the
               GPU's own drift is of the oracle's size, so the tolerance is FACTOR_FP32 x (2 x drift).
  bf16 drift   a bf16 emulation of the oracle -- the weights rounded to bf16, and every convolution's input
               and output rounded to bf16 with fp32 accumulation, as the GPU's bf16 path does (GroupNorm+SiLU
               in fp32 from bf16 values, rounded at the conv input) -- against the fp32 oracle over the whole
               loop. The GPU bf16 path and the emulation are two bf16 evaluations of one fp32 trajectory whose
               rounding points agree (the systematic part -- bf16 weights make a slightly different model --
               is the same for both), so the bf16 x0 bound is FACTOR_BF16 x the emulation's drift; the score
               bound likewise from the emulation's OracleVerifier score differences.

    python tools/derive_tolerances.py [--quick]
"""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ref_cpu as R  # noqa: E402

from itsd.arch import ARCH_A, ARCH_TINY_CFG  # noqa: E402
from itsd.weights import synthetic_state_dict  # noqa: E402

PER = 3 * 32 * 32
STREAM_XT = 0xF0000000
FACTOR_FP32 = 4.0   # 2 fp32 evaluations of one fp64 trajectory, x2 margin
FACTOR_BF16 = 2.0   # two bf16 evaluations of one fp32 trajectory: x2


def _noise_fn(streams):
    def f(step, xx):
        return torch.stack([R.philox_normal(s, step, np.arange(o, o + PER)).reshape(3, 32, 32) for s, o in streams]
                           ).to(xx.dtype)
    return f


def _sd(a, dtype):
    return {k: v.to(dtype) for k, v in synthetic_state_dict(a, 0).items()}


def fp32_vs_fp64(a, x_T, streams, T, beta_T, cfg_labels=None, w=0.0):
    sched = R.schedule(1e-4, beta_T, T)
    out = {}
    for name, dt in (("fp32", torch.float32), ("fp64", torch.float64)):
        sd = _sd(a, dt)
        if cfg_labels is None:
            fw = lambda xx, tt, sd=sd: R.unet_forward(sd, xx, tt, a.ch, a.ch_mult, a.attn, a.num_res_blocks)
        else:
            f3 = lambda xx, tt, ll, sd=sd: R.unet_forward(sd, xx, tt, a.ch, a.ch_mult, a.attn, a.num_res_blocks,
                                                         labels=ll, cfg=True)
            fw = R.cfg_eps(f3, cfg_labels, w)
        t0 = time.time()
        with torch.no_grad():
            out[name] = R.p_sample_loop(fw, x_T.to(dt), sched, _noise_fn(streams)).double()
        print(f"  {name} loop {time.time() - t0:.0f}s", flush=True)
    d = (out["fp32"] - out["fp64"])
    img = d * 0.5  # the saved image x0 * 0.5 + 0.5
    return {"x0_maxabs": d.abs().max().item(), "image_maxabs": img.abs().max().item(),
            "x0_rel_l2": (d.norm() / out["fp64"].norm()).item()}


def _bf(x):
    return x.to(torch.bfloat16).to(torch.float32)


def bf16_emulation(a, x_T, streams, T, beta_T):
    """The fp32 oracle loop and its bf16 emulation (see the module docstring) on the same x_T and noise."""
    import torch.nn.functional as F
    sched = R.schedule(1e-4, beta_T, T)
    sd = _sd(a, torch.float32)
    sdb = {k: (_bf(v) if v.dim() >= 2 else v) for k, v in sd.items()}  # conv / linear weights in bf16
    fw = lambda xx, tt: R.unet_forward(sd, xx, tt, a.ch, a.ch_mult, a.attn, a.num_res_blocks)
    fwb = lambda xx, tt: R.unet_forward(sdb, xx, tt, a.ch, a.ch_mult, a.attn, a.num_res_blocks)
    t0 = time.time()
    with torch.no_grad():
        clean = R.p_sample_loop(fw, x_T, sched, _noise_fn(streams))
    print(f"  fp32 loop {time.time() - t0:.0f}s", flush=True)
    conv2d = F.conv2d
    F.conv2d = lambda x, w, b=None, *args, **kw: _bf(conv2d(_bf(x), w, b, *args, **kw))
    try:
        t0 = time.time()
        with torch.no_grad():
            emu = R.p_sample_loop(fwb, x_T, sched, _noise_fn(streams))
        print(f"  bf16-emulation loop {time.time() - t0:.0f}s", flush=True)
    finally:
        F.conv2d = conv2d
    rel = [((emu[i] - clean[i]).norm() / clean[i].norm()).item() for i in range(x_T.shape[0])]
    dscore = [abs(R.oracle_score(emu[i:i + 1]) - R.oracle_score(clean[i:i + 1])) for i in range(x_T.shape[0])]
    print(f"  bf16 emulation vs fp32: x0 rel-L2 {rel}, score |d| {dscore}", flush=True)
    return {"images": x_T.shape[0], "x0_rel_l2_max": max(rel), "x0_rel_l2_mean": float(np.mean(rel)),
            "score_absdiff_max": max(dscore)}


def bf16_emulation_vs_fixture(name, a, beta_T, w=None):
    """(round 6) C3 / C4: the bf16 emulation's drift over the whole loop against the REFERENCE's own fp32 trajectory
    (tests/golden/full_<name>.npz, tools/gen_golden_full.py: the reference sampler driven with the same Philox
    noise) -- the clean fp32 loop is the fixture, so only the emulation runs here. ConvTranspose2d (the CFG UpSample)
    is rounded like the convolutions."""
    import torch.nn.functional as F
    fx = np.load(os.path.join(ROOT, "tests", "golden", f"full_{name}.npz"))
    x_T, ref = torch.from_numpy(fx["x_T"]), torch.from_numpy(fx["x0"]).double()
    T, seed, rnd, cands = int(fx["T"]), int(fx["seed"]), int(fx["round"]), [int(c) for c in fx["cands"]]
    per = int(np.prod(x_T.shape[1:]))
    run_seed = (seed * 1000003 + rnd) & ((1 << 62) - 1)

    def noise(step, xx):
        return torch.stack([R.philox_normal(run_seed, step, np.arange(i * per, (i + 1) * per)).reshape(x_T.shape[1:])
                            for i in cands])

    sd = _sd(a, torch.float32)
    sdb = {k: (_bf(v) if v.dim() >= 2 else v) for k, v in sd.items()}
    if w is None:
        fwb = lambda xx, tt: R.unet_forward(sdb, xx, tt, a.ch, a.ch_mult, a.attn, a.num_res_blocks)
    else:
        f3 = lambda xx, tt, ll: R.unet_forward(sdb, xx, tt, a.ch, a.ch_mult, a.attn, a.num_res_blocks, labels=ll,
                                               cfg=True)
        fwb = R.cfg_eps(f3, torch.full((len(cands),), int(fx["label"])), w)
    conv2d, convt = F.conv2d, F.conv_transpose2d
    F.conv2d = lambda x, wt, b=None, *args, **kw: _bf(conv2d(_bf(x), wt, b, *args, **kw))
    F.conv_transpose2d = lambda x, wt, b=None, *args, **kw: _bf(convt(_bf(x), wt, b, *args, **kw))
    try:
        t0 = time.time()
        with torch.no_grad():
            raw = R.p_sample_loop(fwb, x_T, R.schedule(1e-4, beta_T, T), noise, clip=False).double()
        print(f"  {name} bf16-emulation loop {time.time() - t0:.0f}s", flush=True)
    finally:
        F.conv2d, F.conv_transpose2d = conv2d, convt
    emu = raw.clamp(-1, 1)
    ref_raw = torch.from_numpy(fx["x0_raw"]).double()
    rel = [((emu[i] - ref[i]).norm() / ref[i].norm()).item() for i in range(len(cands))]
    rel_raw = [((raw[i] - ref_raw[i]).norm() / ref_raw[i].norm()).item() for i in range(len(cands))]
    dscore = [abs(R.oracle_score(emu[i:i + 1].float()) - float(fx["scores"][i])) for i in range(len(cands))]
    print(f"  {name} bf16 emulation vs the reference: x0 rel-L2 {rel}, pre-clip x0 rel-L2 {rel_raw}, score |d| {dscore}",
          flush=True)
    return {"images": len(cands), "against": f"tests/golden/full_{name}.npz (the reference's own fp32 loop)",
            "x0_rel_l2_max": max(rel), "x0_rel_l2_mean": float(np.mean(rel)),
            "raw_rel_l2_max": max(rel_raw), "raw_rel_l2_mean": float(np.mean(rel_raw)),
            "raw_absmax": ref_raw.abs().max().item(), "saturated_frac": (ref.abs() >= 0.999).double().mean().item(),
            "score_absdiff_max": max(dscore)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="short T (smoke of the tool itself)")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "tolerance_derivation.json"))
    ap.add_argument("--only", default="", help="one part (C1c, C1, C2, C5, C3, C4) -> <out>.<part>.json; --merge joins them")
    ap.add_argument("--merge", action="store_true")
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    T = 50 if args.quick else 1000
    res = {"factor_fp32": FACTOR_FP32, "factor_bf16": FACTOR_BF16, "T": T}
    parts = {"C1c": "C1c_cfg_fp32_vs_fp64", "C1": "C1_archA_fp32_vs_fp64", "C2": "C2_bf16_emulation",
             "C5": "C5_bf16_emulation", "C3": "C3_bf16_emulation", "C4": "C4_bf16_emulation"}
    if args.only in ("C2", "C3", "C4", "C5"):  # (round 6) against the reference fixtures of tools/gen_golden_full.py
        if args.only == "C3":
            from itsd.arch import ARCH_C
            r = bf16_emulation_vs_fixture("C3", ARCH_C, 0.028, w=1.8)
        elif args.only == "C4":
            r = bf16_emulation_vs_fixture("C4", dataclasses.replace(ARCH_A, img_size=64), 0.02)
        elif args.only == "C5":
            r = bf16_emulation_vs_fixture("C5", dataclasses.replace(ARCH_A, T=3000), 0.02)
            r["T"] = 3000
        else:
            r = bf16_emulation_vs_fixture("C2", ARCH_A, 0.02)
        with open(f"{args.out}.{args.only}.json", "w") as fh:
            json.dump(r, fh, indent=1)
        return
    if args.merge:
        # parts measured earlier and not re-run keep their recorded values from the existing JSON
        prev = {}
        if os.path.exists(args.out):
            with open(args.out) as fh:
                prev = json.load(fh)
        for k, key in parts.items():
            if os.path.exists(f"{args.out}.{k}.json"):
                with open(f"{args.out}.{k}.json") as fh:
                    res[key] = json.load(fh)
            else:
                res[key] = prev[key]
        _finish(res, args)
        return
    run = lambda k: not args.only or args.only == k
    # C1c: MainCondition eval (tiny CFG UNet, batch 10, w = 1.8, beta_T = 0.028), seed as the GPU test draws it
    a = dataclasses.replace(ARCH_TINY_CFG, T=1000)
    seed = 12345
    x_T = torch.stack([R.philox_normal(seed ^ 0x5A5A, 0, np.arange(j * PER, (j + 1) * PER)).reshape(3, 32, 32)
                       for j in range(10)])
    streams = [(seed, j * PER) for j in range(10)]
    print("C1c tiny CFG fp32 vs fp64", flush=True)
    if run("C1c"):
        res["C1c_cfg_fp32_vs_fp64"] = fp32_vs_fp64(a, x_T, streams, T, 0.028, torch.arange(1, 11), 1.8)
        if args.only:
            with open(f"{args.out}.C1c.json", "w") as fh:
                json.dump(res["C1c_cfg_fp32_vs_fp64"], fh, indent=1)
            return
    # C1: Main.py eval, Arch A, batch 2
    a = ARCH_A
    x_T = torch.stack([R.philox_normal(seed ^ 0xA5A5, 0, np.arange(j * PER, (j + 1) * PER)).reshape(3, 32, 32)
                       for j in range(2)])
    streams = [(seed + 1, j * PER) for j in range(2)]
    print("C1 Arch A fp32 vs fp64", flush=True)
    if run("C1"):
        res["C1_archA_fp32_vs_fp64"] = fp32_vs_fp64(a, x_T, streams, T, 0.02)
        if args.only:
            with open(f"{args.out}.C1.json", "w") as fh:
                json.dump(res["C1_archA_fp32_vs_fp64"], fh, indent=1)
            return
    # C2 / C5: bf16 emulation vs fp32, Arch A, three x_T of the C2 round, at T = 1000 and at T = 3000 (C5)
    x_T = torch.stack([R.philox_normal(21, STREAM_XT, np.arange(i * PER, (i + 1) * PER)).reshape(3, 32, 32)
                       for i in (0, 129, 255)])
    streams = [(77, i * PER) for i in (0, 129, 255)]
    print("C2 bf16 emulation, T=1000", flush=True)
    if run("C2"):
        res["C2_bf16_emulation"] = bf16_emulation(a, x_T, streams, T, 0.02)
        if args.only:
            with open(f"{args.out}.C2.json", "w") as fh:
                json.dump(res["C2_bf16_emulation"], fh, indent=1)
            return
    T5 = 60 if args.quick else 3000
    print("C5 bf16 emulation, T=3000", flush=True)
    if run("C5"):
        res["C5_bf16_emulation"] = bf16_emulation(a, x_T, streams, T5, 0.02)
        res["C5_bf16_emulation"]["T"] = T5
        if args.only:
            with open(f"{args.out}.C5.json", "w") as fh:
                json.dump(res["C5_bf16_emulation"], fh, indent=1)
            return
    _finish(res, args)


def _finish(res, args):
    res["tolerances"] = {
        "FULL_T_FP32_MAXABS": FACTOR_FP32 * 2 * res["C1_archA_fp32_vs_fp64"]["image_maxabs"],
        "FULL_T_FP32_CFG_MAXABS": FACTOR_FP32 * 2 * res["C1c_cfg_fp32_vs_fp64"]["image_maxabs"],
        "FULL_T_BF16_REL_L2": FACTOR_BF16 * res["C2_bf16_emulation"]["x0_rel_l2_max"],
        "FULL_T_BF16_SCORE": FACTOR_BF16 * res["C2_bf16_emulation"]["score_absdiff_max"],
        "C5_BF16_REL_L2": FACTOR_BF16 * res["C5_bf16_emulation"]["x0_rel_l2_max"],
        "C5_BF16_SCORE": FACTOR_BF16 * res["C5_bf16_emulation"]["score_absdiff_max"],
        "FULL_T_BF16_RAW_REL_L2": FACTOR_BF16 * res["C2_bf16_emulation"]["raw_rel_l2_max"],
        "C5_BF16_RAW_REL_L2": FACTOR_BF16 * res["C5_bf16_emulation"]["raw_rel_l2_max"],
        "C3_BF16_RAW_REL_L2": FACTOR_BF16 * res["C3_bf16_emulation"]["raw_rel_l2_max"],
        "C4_BF16_RAW_REL_L2": FACTOR_BF16 * res["C4_bf16_emulation"]["raw_rel_l2_max"],
        "C3_BF16_REL_L2": FACTOR_BF16 * res["C3_bf16_emulation"]["x0_rel_l2_max"],
        "C3_BF16_SCORE": FACTOR_BF16 * res["C3_bf16_emulation"]["score_absdiff_max"],
        "C4_BF16_REL_L2": FACTOR_BF16 * res["C4_bf16_emulation"]["x0_rel_l2_max"],
        "C4_BF16_SCORE": FACTOR_BF16 * res["C4_bf16_emulation"]["score_absdiff_max"],
    }
    res["command"] = ("python tools/derive_tolerances.py --only <part> (C1c, C1, C2, C5, C3, C4), then --merge"
                      + (" --quick" if args.quick else ""))
    print(json.dumps(res, indent=1))
    if not args.quick:
        with open(args.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
