"""Full-length sampled images and scores against the oracle ("Pin full-length sampled
images and scores"; north_star: "sampled images match the reference PyTorch CPU path on fixed seeds
within a stated fp32 tolerance").

One module fixture runs, on the GPU:
  C1   Main.py's eval (config/config.yaml keys through itsd.entry, ``Diffusion/Train.py:808-843``):
       Arch A, T = 1000, fp32 (the reference's precision), synthetic weights, batch_size 1 and 2 --
       the whole ancestral loop ``Diffusion/Diffusion.py:84-102`` in Philox mode;
  C2   one bf16 random-search round of N = 256 Philox candidates at T = 1000 (the bench's round,
       ``search/search_algorithm.py:54-83``) scored by the OracleVerifier (``search/verifier.py:45-66``),
and then the oracle's full 1000-step loop (``oracle.ref_cpu.p_sample_loop``, fp32 CPU) over the two
C1 runs' 3 images and 3 of the 256 candidates (indices 0, 129, 255) in ONE batched loop, each image
fed its own counter-based noise (``R.philox_normal``: the seed the run used, the image's global
element offset), so every comparison is one image's whole trajectory.

Tolerances: DERIVED, not tuned (VERDICT r4 #5c; tools/derive_tolerances.py -> tests/golden/tolerance_derivation.json,
DESIGN.md section 4). Two drifts of the oracle's own whole loop on CPU:
  fp32   the fp32 oracle against the same loop in fp64 (weights, activations, x): the GPU fp32 path and the
         oracle are two fp32 evaluations of one fp64 trajectory, so |GPU - oracle| <= 2 x drift; bound =
         4 x 2 x drift (x2 margin).   C1 Arch A T=1000: drift 6.5e-5 on the saved image -> 5.2e-4;
         C1c tiny CFG w=1.8 T=1000: drift 4.5e-4 -> 3.6e-3.
  bf16   a bf16 emulation of the oracle (weights bf16; every conv's input and output rounded to bf16 with
         fp32 accumulation, as the GPU's bf16 path) against the fp32 oracle: the GPU bf16 path and the
         emulation are two bf16 evaluations of one fp32 trajectory; bound = 2 x the emulation's drift.
         C2 T=1000: x0 rel-L2 3.0e-2 -> 6.1e-2; C5 T=3000: see the JSON (the T=3000 images of the synthetic
         model saturate to +-1, so their rel-L2 counts sign flips: 2 sqrt(k / 3072)).
  scores an exact consequence of the image (_check_score): the search's score equals the verifier on the
         candidate's own x0 (1e-6), and differs from the oracle trajectory's score by at most what the measured
         x0 difference implies (Cauchy-Schwarz on the variance; no sampled bound).
Measured values are printed.
"""
import dataclasses
import json
import os

import numpy as np
import pytest
import torch

from oracle import ref_cpu as R
from itsd import entry as E
from itsd.arch import ARCH_A, ARCH_TINY_CFG
from itsd.diffusion import GaussianDiffusionSampler
from itsd.model import UNet
from itsd.search import SearchEngine
from itsd.verifier import OracleVerifier
from itsd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tolerance_derivation.json")) as _fh:
    _TOL = json.load(_fh)["tolerances"]
FULL_T_FP32_MAXABS = _TOL["FULL_T_FP32_MAXABS"]          # 4 x 2 x the oracle's fp32-vs-fp64 drift (C1)
FULL_T_BF16_REL_L2 = _TOL["FULL_T_BF16_REL_L2"]          # 2 x the bf16 emulation's drift (C2, T = 1000)
FULL_T_BF16_SCORE = _TOL["FULL_T_BF16_SCORE"]
FULL_T_FP32_CFG_MAXABS = _TOL["FULL_T_FP32_CFG_MAXABS"]  # 4 x 2 x the guided loop's fp32-vs-fp64 drift (C1c)
C5_BF16_REL_L2 = _TOL["C5_BF16_REL_L2"]                  # 2 x the bf16 emulation's drift at T = 3000
C5_BF16_SCORE = _TOL["C5_BF16_SCORE"]

T = 1000
PER = 3 * 32 * 32
STREAM_XT = 0xF0000000  # itsd.search._STREAM_XT: candidate x_T of round 0
CANDS = (0, 129, 255)
ENGINE_SEED = 21


def _rel_l2(a, b):
    return (torch.linalg.norm((a - b).flatten()) / torch.linalg.norm(b.flatten())).item()


def _check_score(tag, got_x0, got_score, ref_x0, sampled_bound):
    """The OracleVerifier score of a candidate, in two exact steps (no sampled bound):
    (1) the search's score IS the verifier on the candidate's own image: |score - R.oracle_score(x0)| <= 1e-6;
    (2) against the oracle trajectory's score, the difference the image difference implies: with d = x0 - ref,
        var(ref + d) - var(ref) = 2 cov(ref, d) + var(d) and |cov| <= std(ref) std(d) (Cauchy-Schwarz), and
        1/(1+v1) - 1/(1+v2) = (v2 - v1) / ((1+v1)(1+v2)), so |ds| <= (2 std(ref) std(d) + var(d)) / ((1+v1)(1+v2)).
    The image itself is bounded by the derived rel-L2 tolerance beside this call. (Round 5: the sampled bound
    -- 2 x the largest score drift of 3 bf16-emulation images -- was exceeded at T = 3000, 7.5e-5 vs 6.3e-5, by
    a candidate whose x0 was inside its derived bound: 3 samples do not bound a tail; it is printed, not asserted.)"""
    g, r = got_x0.flatten().double(), ref_x0.flatten().double()
    d = g - r
    self_score = R.oracle_score(got_x0.unsqueeze(0).float())
    assert abs(float(got_score) - self_score) <= 1e-6, (tag, float(got_score), self_score)
    v1, v2 = torch.var(r).item(), torch.var(g).item()
    implied = (2 * torch.std(r).item() * torch.std(d).item() + torch.var(d).item()) / ((1 + v1) * (1 + v2))
    s_ref = R.oracle_score(ref_x0.unsqueeze(0))
    ds = abs(float(got_score) - s_ref)
    print(f"{tag}: score {float(got_score):.6f} (verifier on its own x0 {self_score:.6f}) vs oracle {s_ref:.6f}: "
          f"|d| {ds:.2e}, implied by the x0 difference <= {implied:.2e} (sampled emulation figure {sampled_bound:.2e})")
    assert ds <= implied * (1 + 1e-6) + 1e-7


@pytest.fixture(scope="module")
def full_T(tmp_path_factory):
    out = {}
    # ---- C1: Main.py eval, batch_size 1 and 2 (fp32, T = 1000, Philox seed drawn by the sampler)
    c1 = []
    for bs, seed in ((1, 7), (2, 8)):
        d = tmp_path_factory.mktemp(f"c1_bs{bs}")
        cfg = E.load_config(None, ["weights=random", f"batch_size={bs}", "inference_T=1000", f"sampled_dir={d}",
                                   f"seed={seed}", "nrow=8", "img_size=32"])
        res = E.run(cfg)
        assert res["sampler_seed"] is not None
        c1.append({"x_T": res["noisy"].cpu(), "sampled": res["sampled"].cpu(), "seed": int(res["sampler_seed"])})
        torch.cuda.empty_cache()
    out["c1"] = c1
    # ---- C2: a bf16 N = 256 Philox round (the bench's round protocol)
    a = ARCH_A
    net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=32, precision="bf16").to("cuda:0")
    net.load_state_dict(synthetic_state_dict(a, 0))
    smp = GaussianDiffusionSampler(net, 1e-4, 0.02, T)
    eng = SearchEngine(smp, OracleVerifier(), seed=ENGINE_SEED)
    r = eng.run_round(0, 256, (1, 3, 32, 32))
    run_seed = (ENGINE_SEED * 1000003 + 0) & ((1 << 62) - 1)  # SearchEngine.run_round's sampler key
    out["c2"] = {"x0": r.local_images.cpu(), "scores": r.scores.clone(), "run_seed": run_seed}
    del eng, smp, net
    torch.cuda.empty_cache()
    # ---- the oracle: one batched fp32 loop over the 6 images, each with its own noise stream
    x_T, streams = [], []  # streams[i] = (seed, first global element of image i)
    for run in c1:
        for j in range(run["x_T"].shape[0]):
            x_T.append(run["x_T"][j])
            streams.append((run["seed"], j * PER))
    for i in CANDS:
        x_T.append(R.philox_normal(ENGINE_SEED, STREAM_XT, np.arange(i * PER, (i + 1) * PER)).reshape(3, 32, 32))
        streams.append((run_seed, i * PER))
    x_T = torch.stack(x_T)

    def noise(step, xx):
        return torch.stack([R.philox_normal(s, step, np.arange(o, o + PER)).reshape(3, 32, 32) for s, o in streams])

    sd = synthetic_state_dict(a, 0)
    fw = lambda xx, tt: R.unet_forward(sd, xx, tt, a.ch, a.ch_mult, a.attn, a.num_res_blocks)
    with torch.no_grad():
        out["oracle_x0"] = R.p_sample_loop(fw, x_T, R.schedule(1e-4, 0.02, T), noise)
    out["oracle_x_T"] = x_T
    return out


def test_C1_main_eval_T1000_fp32_vs_oracle(full_T):
    """Main.py's eval end to end at the reference's precision: the saved image (x0 * 0.5 + 0.5) of
    batch_size 1 and 2 against the oracle's full 1000-step loop on the same x_T and noise."""
    ref = full_T["oracle_x0"] * 0.5 + 0.5
    k = 0
    for run in full_T["c1"]:
        n = run["sampled"].shape[0]
        d = (run["sampled"] - ref[k:k + n]).abs().max().item()
        rel = _rel_l2(run["sampled"] * 2 - 1, full_T["oracle_x0"][k:k + n])
        print(f"C1 batch {n}: full T=1000 fp32 x0 max|d| = {d:.3e} (rel-L2 of x0 {rel:.3e})")
        assert d <= FULL_T_FP32_MAXABS
        k += n


def test_C2_bf16_round_T1000_candidates_and_scores_vs_oracle(full_T):
    """Three candidates of one bf16 N = 256 round: the denoised x0 (rel-L2) and the OracleVerifier
    score the search prunes on, against the fp32 oracle's full loop and R.oracle_score."""
    c2 = full_T["c2"]
    for k, i in enumerate(CANDS):
        # the round's x_T is the Philox generator's (itsd_noise == R.philox_normal is pinned by
        # test_gpu_search.test_philox_noise_kernel_matches_oracle), so the oracle started from it
        ref = full_T["oracle_x0"][3 + k]
        got = c2["x0"][i]
        rel = _rel_l2(got, ref)
        print(f"C2 bf16 candidate {i}: x0 rel-L2 {rel:.3e}, max|d| {(got - ref).abs().max().item():.3e}")
        assert rel <= FULL_T_BF16_REL_L2
        _check_score(f"C2 candidate {i}", got, c2["scores"][i], ref, FULL_T_BF16_SCORE)


C5_T, C5_N, C5_CANDS, C5_SEED = 3000, 128, (0, 64, 127), 33
STREAM_PERTURB = 0xE0000000  # itsd.search._STREAM_PERTURB: perturbed candidates (pivot + scale z) of round 0


def test_C5_path_search_round_T3000_candidates_and_scores_vs_oracle():
    """C5 at full length (VERDICT r4 #5a): one bf16 path-search round (``search/search_algorithm.py:265-336``;
    candidates = pivot + 0.1 z) of the bench shard N = 128 over the whole T = 3000 schedule of
    ``fine_tune_extended_T.py`` (betas 1e-4 .. 0.02), three candidates (0, 64, 127) -- the denoised x0 and the
    OracleVerifier score the search prunes on -- against the oracle's full 3000-step fp32 loop on the same
    x_T and Philox noise. Bounds: C5_BF16_REL_L2 / C5_BF16_SCORE, derived (tests/golden/tolerance_derivation.json)."""
    a = dataclasses.replace(ARCH_A, T=C5_T)
    net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=32, precision="bf16").to("cuda:0")
    net.load_state_dict(synthetic_state_dict(a, 0))
    smp = GaussianDiffusionSampler(net, 1e-4, 0.02, C5_T)
    eng = SearchEngine(smp, OracleVerifier(), seed=C5_SEED)
    shape = (1, 3, 32, 32)
    pivot = eng.initial_noise(shape)
    r = eng.run_round(0, C5_N, shape, pivot=pivot, scale=0.1, kind="path")
    run_seed = (C5_SEED * 1000003 + 0) & ((1 << 62) - 1)
    # the candidates' x_T regenerated on the device (the same kernel, bit-identical) -> the oracle's start
    x_T = torch.cat([eng.candidate_noise(0, i, 1, shape, pivot=pivot, scale=0.1) for i in C5_CANDS]).cpu()
    x0 = r.local_images.cpu()
    scores = r.scores.clone()
    del eng, smp, net
    torch.cuda.empty_cache()
    streams = [(run_seed, i * PER) for i in C5_CANDS]

    def noise(step, xx):
        return torch.stack([R.philox_normal(sd_, step, np.arange(o, o + PER)).reshape(3, 32, 32) for sd_, o in streams])

    sd = synthetic_state_dict(a, 0)
    fw = lambda xx, tt: R.unet_forward(sd, xx, tt, a.ch, a.ch_mult, a.attn, a.num_res_blocks)
    with torch.no_grad():
        ref = R.p_sample_loop(fw, x_T, R.schedule(1e-4, 0.02, C5_T), noise)
    for k, i in enumerate(C5_CANDS):
        rel = _rel_l2(x0[i], ref[k])
        print(f"C5 bf16 path candidate {i}: T=3000 x0 rel-L2 {rel:.3e}, max|d| {(x0[i] - ref[k]).abs().max().item():.3e}")
        assert rel <= C5_BF16_REL_L2
        _check_score(f"C5 candidate {i}", x0[i], scores[i], ref[k], C5_BF16_SCORE)


def test_C1c_main_condition_eval_T1000_fp32_vs_oracle(tmp_path):
    """MainCondition.py's eval (``TrainCondition.py:118-151`` through ``itsd.entry`` with
    config/condition_config.yaml keys): the class-block labels of batch_size 10, guided sampling
    with w = 1.8 and beta_T = 0.028 over T = 1000 steps in fp32 (the tiny CFG UNet: channel 32,
    channel_mult [1, 2], 1 ResBlock a level, synthetic weights), the saved image against the oracle's
    full guided loop (``DiffusionCondition.py:79-105``: eps = (1 + w) eps(labels) - w eps(0)) on the
    same x_T and Philox noise: max|d| <= FULL_T_FP32_CFG_MAXABS (derived: 4 x 2 x the guided loop's own
    fp32-vs-fp64 drift, 4.5e-4 -- the guidance weights 2.8 / 1.8 amplify sum-order differences; measured
    5.0e-4 in round 4)."""
    a = dataclasses.replace(ARCH_TINY_CFG, T=1000)
    cfg = E.load_config(None, ["weights=random", "T=1000", "channel=32", "channel_mult=[1,2]", "num_res_blocks=1",
                               "batch_size=10", f"sampled_dir={tmp_path}", "seed=11", "nrow=5"],
                        config_name="condition_config")
    res = E.run(cfg, condition=True)
    labels = res["labels"].cpu()
    assert labels.tolist() == list(range(1, 11))
    seed = int(res["sampler_seed"])
    x_T = res["noisy"].cpu()
    sd = synthetic_state_dict(a, 0)
    fw = lambda xx, tt, ll: R.unet_forward(sd, xx, tt, a.ch, a.ch_mult, a.attn, a.num_res_blocks, labels=ll, cfg=True)
    n = x_T.shape[0]

    def noise(step, xx):
        return torch.stack([R.philox_normal(seed, step, np.arange(j * PER, (j + 1) * PER)).reshape(3, 32, 32)
                            for j in range(n)])

    with torch.no_grad():
        ref = R.p_sample_loop(R.cfg_eps(fw, labels, float(cfg["w"])), x_T, R.schedule(1e-4, 0.028, 1000), noise)
    d = (res["sampled"].cpu() - (ref * 0.5 + 0.5)).abs().max().item()
    print(f"C1c MainCondition eval, batch 10, T=1000 fp32: x0 max|d| {d:.3e}")
    assert d <= FULL_T_FP32_CFG_MAXABS
