"""GPU parity: the HIP path (through the C ABI) vs the reference-pinned fixtures and
the CPU oracle on the same seeded inputs.

Tolerances ("Parity"):
  fp32 mode  per-forward eps   max|d| <= 2e-4          (f32 MFMA, different summation order)
             trajectories x0   max|d| <= 2e-3          (T <= 20, injected reference noise)
  bf16 mode  per-forward eps   rel-L2  <= 2e-2
  verifiers                    |d| <= 1e-5 (NaN where the reference gives NaN)
"""
import math

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref_cpu as R
import dataclasses

from itsd.arch import ARCH_A, ARCH_C, ARCH_TINY, ARCH_TINY_CFG
from itsd.diffusion import CondGaussianDiffusionSampler, GaussianDiffusionSampler, reference_noise_plan
from itsd.model import CondUNet, UNet
from itsd.search import SearchEngine
from itsd.verifier import AestheticPredictor, OracleVerifier, SelfSupervisedVerifier
from itsd.weights import synthetic_state_dict
from itsd import runtime as rt

pytestmark = pytest.mark.gpu

EPS_TOL_FP32 = 2e-4
TRAJ_TOL_FP32 = 2e-3
REL_L2_BF16 = 2e-2


def _net(a, precision="fp32", seed=0):
    if a.cfg:
        net = CondUNet(a.T, a.num_labels, a.ch, a.ch_mult, a.num_res_blocks, 0.0, img_size=a.img_size,
                       precision=precision)
    else:
        net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=a.img_size, precision=precision)
    net.load_state_dict(synthetic_state_dict(a, seed))
    return net.to("cuda:0")


def _oracle(a, sd):
    return lambda x, t, labels=None: R.unet_forward(sd, x, t, a.ch, a.ch_mult, a.attn, a.num_res_blocks,
                                                    labels=labels, cfg=a.cfg)


def _rel_l2(a, b):
    return (torch.linalg.norm((a - b).flatten()) / torch.linalg.norm(b.flatten())).item()


def test_native_lib_is_loaded(gpu_lib):
    assert gpu_lib.itsd_version() == 1


@pytest.mark.parametrize("arch,fix", [(ARCH_TINY, "tiny_ddpm_eps"), (ARCH_A, "archA_eps")])
def test_forward_fp32_vs_reference(arch, fix):
    g = golden(fix)
    net = _net(arch)
    eps = net(torch.from_numpy(g["x"]).cuda(), torch.from_numpy(g["t"]).cuda()).cpu().numpy()
    np.testing.assert_allclose(eps, g["eps"], atol=EPS_TOL_FP32, rtol=0)


def test_forward_cfg_fp32_vs_reference():
    g = golden("tiny_cfg_eps")
    net = _net(ARCH_TINY_CFG)
    eps = net(torch.from_numpy(g["x"]).cuda(), torch.from_numpy(g["t"]).cuda(),
              torch.from_numpy(g["labels"]).cuda()).cpu().numpy()
    np.testing.assert_allclose(eps, g["eps"], atol=EPS_TOL_FP32, rtol=0)


@pytest.mark.parametrize("n", [1, 3, 8])
def test_forward_bf16_archA_vs_oracle(n):
    a = ARCH_A
    sd = synthetic_state_dict(a, 0)
    net = _net(a, "bf16")
    gen = torch.Generator().manual_seed(n)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, 1000, (n,), generator=gen)
    eps = net(x.cuda(), t.cuda()).cpu()
    with torch.no_grad():
        ref = _oracle(a, sd)(x, t)
    assert _rel_l2(eps, ref) < REL_L2_BF16


ARCH_A64 = dataclasses.replace(ARCH_A, img_size=64)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("arch,fix", [(ARCH_C, "archC_eps"), (ARCH_A64, "archA64_eps")])
def test_forward_full_configs_vs_reference(arch, fix, precision):
    """C3 (CFG UNet, flash attention at S = 1024 in bf16) and C4 (Arch A at 64 px)
    against reference outputs: fp32 max-abs, bf16 relative L2."""
    g = golden(fix)
    net = _net(arch, precision)
    args = [torch.from_numpy(g["x"]).cuda(), torch.from_numpy(g["t"]).cuda()]
    if arch.cfg:
        args.append(torch.from_numpy(g["labels"]).cuda())
    eps = net(*args).cpu()
    ref = torch.from_numpy(g["eps"])
    if precision == "fp32":
        np.testing.assert_allclose(eps.numpy(), ref.numpy(), atol=EPS_TOL_FP32, rtol=0)
    else:
        assert _rel_l2(eps, ref) < REL_L2_BF16


def test_trajectory_tiny_fp32_vs_reference():
    g = golden("tiny_ddpm_traj")
    T = int(g["T"])
    net = _net(ARCH_TINY)
    smp = GaussianDiffusionSampler(net, 1e-4, 0.02, T)
    noise = torch.cat([torch.zeros(1, 2, 3, 32, 32), torch.from_numpy(g["noise"]).flip(0)])  # [T] by step t
    for graph in (True, False):
        x0 = smp(torch.from_numpy(g["x_T"]).cuda(), noise=noise, graph=graph).cpu().numpy()
        np.testing.assert_allclose(x0, g["x0"], atol=TRAJ_TOL_FP32, rtol=0)


def test_trajectory_cfg_fp32_vs_reference():
    g = golden("tiny_cfg_traj")
    T = int(g["T"])
    net = _net(ARCH_TINY_CFG)
    smp = CondGaussianDiffusionSampler(net, 1e-4, 0.028, T, w=float(g["w"]))
    noise = torch.cat([torch.zeros(1, 2, 3, 32, 32), torch.from_numpy(g["noise"]).flip(0)])
    x0 = smp(torch.from_numpy(g["x_T"]).cuda(), torch.from_numpy(g["labels"]).cuda(), noise=noise).cpu().numpy()
    np.testing.assert_allclose(x0, g["x0"], atol=TRAJ_TOL_FP32, rtol=0)


def test_trajectory_cfg_bf16_vs_reference():
    """Guided bf16 sampler (cond || uncond batch through the MFMA tail with the fused
    tail GroupNorm) against the reference trajectory: relative L2 <= 3e-2 after T = 6."""
    g = golden("tiny_cfg_traj")
    T = int(g["T"])
    net = _net(ARCH_TINY_CFG, "bf16")
    smp = CondGaussianDiffusionSampler(net, 1e-4, 0.028, T, w=float(g["w"]))
    noise = torch.cat([torch.zeros(1, 2, 3, 32, 32), torch.from_numpy(g["noise"]).flip(0)])
    x0 = smp(torch.from_numpy(g["x_T"]).cuda(), torch.from_numpy(g["labels"]).cuda(), noise=noise).cpu()
    assert _rel_l2(x0, torch.from_numpy(g["x0"])) < 3e-2


def test_trajectory_archA_fp32_vs_reference():
    g = golden("archA_traj")
    T = int(g["T"])
    torch.manual_seed(int(g["seed"]))
    x_T, noise = reference_noise_plan((2, 3, 32, 32), T, n_runs=1)
    net = _net(ARCH_A)
    smp = GaussianDiffusionSampler(net, 1e-4, 0.02, T)
    x0 = smp(x_T[0].cuda(), noise=noise).cpu().numpy()
    np.testing.assert_allclose(x0, g["x0"], atol=TRAJ_TOL_FP32, rtol=0)


def test_verifiers_vs_reference():
    g = golden("verifiers")
    for case in ("b1_neg", "b4_neg", "b4_pos", "b2_neg"):
        im = torch.from_numpy(g[case + "_images"]).cuda()
        for name, V in (("oracle", OracleVerifier()), ("selfsup", SelfSupervisedVerifier()),
                        ("aesthetic", AestheticPredictor())):
            want = float(g[f"{case}_{name}"])
            got = V.score(im)
            if math.isnan(want):
                assert math.isnan(got), (case, name)
            else:
                assert abs(got - want) <= 1e-5, (case, name, got, want)


def test_verifier_branches_vs_reference():
    """The two verifier branches off the search path run natively too: OracleVerifier with
    dataset stats (ITSD_VERIFY_MEAN, verifier.py:66) and the paired SelfSupervisedVerifier
    (itsd_verify_paired, verifier.py:235-240), vs the reference's outputs."""
    g = golden("verifier_branches")
    ov = OracleVerifier(dataset_stats={"mu": np.zeros(4), "sigma": np.eye(4)})
    for case in ("b1", "b3", "b2_64"):
        got = ov.score(torch.from_numpy(g[case + "_images"]).cuda())
        assert abs(got - float(g[case + "_oracle_stats"])) <= 1e-6, case
    sv = SelfSupervisedVerifier()
    for case in ("p32", "p64"):
        got = sv.score(torch.from_numpy(g[case + "_images"]).cuda(), reference_features=torch.from_numpy(g[case + "_ref"]))
        assert abs(got - float(g[case + "_paired"])) <= 1e-6, case
    with pytest.raises(RuntimeError):  # the reference's .item() of a 2-vector
        sv.score(torch.zeros(2, 3, 32, 32).cuda(), reference_features=torch.zeros(2, 192))


def test_verifier_batched_equals_per_candidate():
    gen = torch.Generator().manual_seed(9)
    im = (torch.randn(12, 3, 32, 32, generator=gen) * 0.5).clamp(-1, 1)
    im[8:] = im[8:].abs()  # candidates without negatives take the other aesthetic branch
    for V in (OracleVerifier(), SelfSupervisedVerifier(), AestheticPredictor()):
        batch = V.score_batch(im.cuda(), 4).cpu()
        for c in range(4):
            ref = R.VERIFIERS[{0: "oracle", 1: "selfsup", 2: "aesthetic"}[V.kind]](im[3 * c:3 * c + 3])
            assert abs(batch[c].item() - ref) <= 1e-5


def test_search_outcomes_match_reference_T5():
    """RandomSearch / ZeroOrder / PathSearch on the tiny UNet, T=5, seeds of the golden
    run: candidates batched into one native sampler run with the reference's noise."""
    g = golden("search_T5")
    T = 5
    net = _net(ARCH_TINY)
    smp = GaussianDiffusionSampler(net, 1e-4, 0.02, T)
    ver = OracleVerifier()
    shape = (1, 3, 32, 32)

    # RandomSearch(4): per candidate randn(noise) then T-1 step draws (search_algorithm.py:65-75)
    torch.manual_seed(0)
    x_T, noise = reference_noise_plan(shape, T, n_runs=4)
    x = smp(x_T.reshape(4, 3, 32, 32).cuda(), noise=noise)
    scores = ver.score_batch(x, 4).cpu().numpy()
    np.testing.assert_allclose(scores, g["random_scores"], atol=1e-5)
    assert int(np.argmax(scores)) == int(np.argmax(g["random_scores"]))
    np.testing.assert_array_equal(x_T[int(np.argmax(scores))].numpy(), g["random_best_noise"])

    # ZeroOrder(3 neighbours, 2 iterations): neighbours drawn first, then each one's T-1 draws
    torch.manual_seed(1)
    pivot = torch.randn(shape)
    best_score, best_noise = float("-inf"), pivot
    for it in range(2):
        neigh = torch.stack([pivot + torch.randn_like(pivot) * (1 - 0.95) for _ in range(3)])
        zs = []
        for _ in range(3):
            zs.append(torch.stack([torch.randn(shape) for _ in range(T - 1)] + [torch.zeros(shape)]).flip(0))
        noise = torch.stack(zs, dim=1).reshape(T, 3, 3, 32, 32)
        x = smp(neigh.reshape(3, 3, 32, 32).cuda(), noise=noise)
        sc = ver.score_batch(x, 3).cpu().numpy()
        np.testing.assert_allclose(sc, g["zo_scores"][it], atol=1e-5)
        if sc.max() > best_score:  # search_algorithm.py:193-196
            best_score, best_noise = float(sc.max()), neigh[int(np.argmax(sc))]
            pivot = best_noise
    np.testing.assert_allclose(best_noise.numpy(), g["zo_best_noise"], atol=1e-6)
    assert abs(best_score - float(g["zo_best_score"])) < 1e-5


def test_noise_generator_statistics_and_sharding():
    out = torch.empty(64, 3, 32, 32, device="cuda")
    rt.noise(out, 64, seed=123, stream_id=7)
    z = out.cpu()
    assert abs(z.mean().item()) < 0.01 and abs(z.std().item() - 1) < 0.01
    # candidate noise depends only on its global index: a shard regenerates the same values
    part = torch.empty(16, 3, 32, 32, device="cuda")
    rt.noise(part, 16, seed=123, stream_id=7, cand_offset=32)
    assert torch.equal(part.cpu(), z[32:48])


def test_batch_invariance_and_sampler_determinism_bf16():
    """A candidate's trajectory is a function of (seed, global index) only: running it
    in a batch of 8 or as the second shard of 4 gives bit-identical results."""
    a = ARCH_TINY
    net = _net(a, "bf16")
    smp = GaussianDiffusionSampler(net, 1e-4, 0.02, 1000)
    x = torch.empty(8, 3, 32, 32, device="cuda")
    rt.noise(x, 8, seed=5, stream_id=0xF0000000)
    full = smp.run(x.clone(), t_begin=999, t_end=990, seed=77)
    per = x[0].numel()
    half = smp.run(x[4:].clone(), t_begin=999, t_end=990, seed=77, noise_offset=4 * per)
    assert torch.equal(full[4:], half)
    again = smp.run(x.clone(), t_begin=999, t_end=990, seed=77, graph=False)
    assert torch.equal(full, again)


def test_engine_random_search_full_T_archA_bf16():
    """The benchmark path at small N: 8 candidates x T=1000 on Arch A in bf16; finite,
    clipped, and the reported best is the argmax of the scores."""
    net = _net(ARCH_A, "bf16")
    smp = GaussianDiffusionSampler(net, 1e-4, 0.02, 1000)
    eng = SearchEngine(smp, OracleVerifier(), seed=1)
    best_noise, best_score, info = eng.random_search(8, (1, 3, 32, 32))
    sc = torch.tensor(info["scores"], dtype=torch.float64)
    assert torch.isfinite(sc).all()
    assert best_score == sc.max().item() and info["best_index"] == int(torch.argmax(sc))
    assert best_noise.shape == (1, 3, 32, 32)


def _attn_ref(qkv):
    """Plain PyTorch fp32 AttnBlock core (Model.py:152-161)."""
    q, k, v = qkv.float().chunk(3, dim=2)
    w = torch.bmm(q, k.transpose(1, 2)) * (q.shape[2] ** -0.5)
    return torch.bmm(torch.softmax(w, dim=-1), v)


@pytest.mark.parametrize("n,S,C,dtype,with_vt,wide", [
    (2, 256, 384, torch.bfloat16, True, 1),   # Arch A at 64 px, level 2 (C4): channel-split kernel
    (3, 256, 512, torch.bfloat16, True, 1),   # C3 level 1: channel-split kernel
    (2, 1024, 256, torch.bfloat16, True, 2),  # channel-split forced where the flash kernel runs
    (2, 64, 256, torch.bfloat16, True, 2),    # channel-split forced at S = 64
    (2, 1024, 128, torch.bfloat16, True, 1),  # C3 level 0: flash kernel
    (1, 4096, 256, torch.bfloat16, True, 1),  # Arch A at 256 px, level 2: flash kernel
    (3, 320, 64, torch.bfloat16, True, 1),    # flash kernel, ragged last query tile
    (2, 64, 384, torch.bfloat16, True, 1),    # Arch A level 2: whole-row MFMA kernel
    (2, 64, 1024, torch.bfloat16, True, 1),   # C3 level 2: channel-split kernel, 8 waves a query group
    (3, 128, 1024, torch.bfloat16, True, 1),  # the same, 4 key tiles
    (2, 64, 1024, torch.bfloat16, True, 0),   # C3 level 2 on the whole-row MFMA kernel
    (2, 16, 1024, torch.bfloat16, True, 1),   # C3 level 3
    (2, 4, 512, torch.bfloat16, False, 1),    # C3 level 4: VALU kernel
    (2, 1024, 128, torch.float32, False, 1),  # parity mode
    (3, 1, 256, torch.float32, False, 1),     # C3 level 5 (S = 1: softmax of one key)
])
def test_attention_kernels_vs_torch(n, S, C, dtype, with_vt, wide):
    gen = torch.Generator().manual_seed(S + C)
    qkv = (torch.randn(n, S, 3 * C, generator=gen) * 1.5).to(dtype)
    ref = _attn_ref(qkv)
    d = qkv.cuda()
    vt = d[:, :, 2 * C:].transpose(1, 2).contiguous() if with_vt else None
    rt.set_option("attn_wide", wide)
    try:
        out = rt.attention(d, vt).float().cpu()
        assert torch.equal(out, rt.attention(d, vt).float().cpu())  # deterministic
    finally:
        rt.set_option("attn_wide", 1)
    if dtype == torch.float32:
        np.testing.assert_allclose(out.numpy(), ref.numpy(), atol=5e-5, rtol=0)  # fp32, S-term sums
    else:  # P and the output are rounded to bf16
        assert _rel_l2(out, ref) < 1e-2
        assert (out - ref).abs().max().item() < 3e-2 * ref.abs().max().item()


@pytest.mark.parametrize("S,C", [(256, 384), (256, 512), (1024, 256)])
def test_channel_split_attention_query_groups_bit_identical(S, C):
    """attn_cs_kernel with 2 query groups a block (512 threads) computes every query exactly as with one
    (the same wave-level products and partial-score order): bit-identical outputs, and within the bf16
    bound of the fp32 reference."""
    n = 3
    gen = torch.Generator().manual_seed(7 * S + C)
    qkv = (torch.randn(n, S, 3 * C, generator=gen) * 1.5).to(torch.bfloat16)
    d = qkv.cuda()
    vt = d[:, :, 2 * C:].transpose(1, 2).contiguous()
    outs = []
    rt.set_option("attn_wide", 2)
    try:
        for nq in (1, 2):
            rt.set_option("attn_wide_nq", nq)
            outs.append(rt.attention(d, vt).float().cpu())
    finally:
        rt.set_option("attn_wide", 1)
        rt.set_option("attn_wide_nq", 1)
    assert torch.equal(outs[0], outs[1])
    assert _rel_l2(outs[1], _attn_ref(qkv)) < 1e-2


_TILE_DEFAULTS = {"gn_wide": 1, "splitk": 1, "p4_sub": 1}


def _eps_with(net, x, t, **opts):
    """eps of one forward under itsd_set_option overrides (the defaults restored after)."""
    try:
        for k, v in opts.items():
            rt.set_option(k, v)
        return net(x, t).cpu()
    finally:
        for k, v in _TILE_DEFAULTS.items():
            rt.set_option(k, v)


@pytest.mark.parametrize("n", [8, 12])
def test_persistent_vs_128px_fused_convs_and_oracle(n):
    """The shipped persistent fused conv (conv3x3_gn_p4_kernel, forced on with gn_wide=2) against
    the 128-pixel fused conv (conv3x3_gn_kernel, gn_wide=0; the bit-identity anchor of the
    earlier 256-pixel generations, which now live in diagnostic builds only): each is
    deterministic run to run, within 1.5e-2 relative L2 of the other (the persistent kernel sums
    the consumer GroupNorm statistics in another fixed order; fp32 statistics that differ in the
    last bits flip bf16 roundings downstream; measured 0.6-1.0e-2, the size of the bf16-vs-fp32
    gap itself) and within the bf16 tolerance of the oracle, with and without split-K."""
    a = ARCH_A
    net = _net(a, "bf16")
    gen = torch.Generator().manual_seed(200 + n)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, 1000, (n,), generator=gen)
    xd, td = x.cuda(), t.cuda()
    narrow = _eps_with(net, xd, td, gn_wide=0, splitk=0)
    assert torch.equal(narrow, _eps_with(net, xd, td, gn_wide=0, splitk=0))
    p4 = _eps_with(net, xd, td, gn_wide=2, splitk=0)
    assert torch.equal(p4, _eps_with(net, xd, td, gn_wide=2, splitk=0))
    with torch.no_grad():
        ref = _oracle(a, synthetic_state_dict(a, 0))(x, t)
    print(f"rel-L2 vs oracle: 128-px {_rel_l2(narrow, ref):.3e} persistent {_rel_l2(p4, ref):.3e}; "
          f"persistent vs 128-px {_rel_l2(p4, narrow):.3e}")
    assert _rel_l2(p4, narrow) < 1.5e-2
    assert _rel_l2(narrow, ref) < REL_L2_BF16 and _rel_l2(p4, ref) < REL_L2_BF16
    p4_sk = _eps_with(net, xd, td, gn_wide=2, splitk=1)
    assert _rel_l2(p4_sk, ref) < REL_L2_BF16


def test_persistent_vs_128px_fused_convs_full_batch():
    """At the bench batch (N = 256, where the automatic choice takes the persistent kernel with
    several tiles per block) the shipped forward is within 1.5e-2 relative L2 of the 128-pixel
    kernels' forward and within the oracle's bf16 tolerance on a sample of the batch."""
    net = _net(ARCH_A, "bf16")
    gen = torch.Generator().manual_seed(3)
    xc = torch.randn(256, 3, 32, 32, generator=gen)
    tc = torch.randint(0, 1000, (256,), generator=gen)
    x, t = xc.cuda(), tc.cuda()
    narrow = _eps_with(net, x, t, gn_wide=0, splitk=0)
    auto = _eps_with(net, x, t)
    assert torch.isfinite(auto).all() and _rel_l2(auto, narrow) < 1.5e-2
    with torch.no_grad():
        ref = _oracle(ARCH_A, synthetic_state_dict(ARCH_A, 0))(xc[:4], tc[:4])
    assert _rel_l2(auto[:4], ref) < REL_L2_BF16


def test_persistent_fused_convs_cfg():
    """CFG UNet (C3 arch, 512-channel 16x16 level: four cout tiles, cond_proj rows in the
    epilogue) on the reference fixture input: persistent kernel forced on vs the 128-pixel
    kernels and vs the reference's eps."""
    g = golden("archC_eps")
    net = _net(ARCH_C, "bf16")
    x, t, lab = (torch.from_numpy(g[k]).cuda() for k in ("x", "t", "labels"))
    outs = []
    for opts in ({"gn_wide": 0, "splitk": 0}, {"gn_wide": 2}):
        try:
            for k, v in opts.items():
                rt.set_option(k, v)
            outs.append(net(x, t, lab).cpu())
        finally:
            for k, v in _TILE_DEFAULTS.items():
                rt.set_option(k, v)
    assert _rel_l2(outs[1], outs[0]) < 1.5e-2
    for o in outs:
        assert _rel_l2(o, torch.from_numpy(g["eps"])) < REL_L2_BF16


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_subpixel_upsample_convs_at_every_level(precision):
    """Every nearest-x2 upsample conv of Arch A runs as 4 sub-pixel 2x2 phase GEMMs (linear
    addressing), including the 8x8 / 16x16 outputs whose phase images are smaller than a
    128-pixel tile: those keep one GroupNorm statistics slot per (image, phase), and the
    following GroupNorms sum them (per-tensor slot counts). The forward stays on the oracle."""
    a = ARCH_A
    net = _net(a, precision)
    n = 3
    gen = torch.Generator().manual_seed(71)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, 1000, (n,), generator=gen)
    ops = net.native(n).profile_ops(x.cuda(), t.cuda().to(torch.int32))
    ups = [o for o in ops if o["kind"] == "conv" and o["stride_up"] == 11]
    assert len(ups) == 3, [o["H"] for o in ups]
    for o in ups:  # conv_pipe<T, 2, true>: the linear (sub-pixel) variant; <.., false> is the 9-tap gather
        assert "true" in o["kernel"], (o["H"], o["kernel"])
    eps = net(x.cuda(), t.cuda()).cpu()
    with torch.no_grad():
        ref = _oracle(a, synthetic_state_dict(a, 0))(x, t)
    if precision == "fp32":
        assert (eps - ref).abs().max().item() < 2e-4
    else:
        assert _rel_l2(eps, ref) < REL_L2_BF16


@pytest.mark.parametrize("n", [32, 64, 256])  # (n = 32: the 8x8 -> 16x16 launch's 96 tiles, on p4 since round 6)
def test_p4_subpixel_upsample_convs_vs_conv_pipe_and_oracle(n):
    """The 16x16 -> 32x32 and 8x8 -> 16x16 nearest-x2 upsample convs (Model.py:121-126) on
    conv3x3_gn_p4_kernel's sub-pixel form (AB = 128: 4 phases x 256 input-grid pixels x 128 couts per
    tile, the phase's 2x2 folded taps, outputs scattered to (2i + py, 2j + px), one GroupNorm statistics
    slot per (image, phase, 128 pixels)) against the same GEMMs on conv_pipe (p4_sub = 0; the k order
    differs: chunk-major vs tap-major): deterministic, within 1e-2 relative L2 of each other and within
    the bf16 bound of the oracle. (The 4x4 -> 8x8 upsample stays on conv_pipe: p4 has no 4x4 form.)"""
    a = ARCH_A
    net = _net(a, "bf16")
    gen = torch.Generator().manual_seed(500 + n)
    xc = torch.randn(n, 3, 32, 32, generator=gen)
    tc = torch.randint(0, 1000, (n,), generator=gen)
    x, t = xc.cuda(), tc.cuda()
    ops = net.native(n).profile_ops(x, t.to(torch.int32))
    ups = {o["H"]: o["kernel"] for o in ops if o["kind"] == "conv" and o["stride_up"] == 11}
    assert "conv3x3_gn_p4_kernel<16, 128>" in ups[32] and "conv3x3_gn_p4_kernel<8, 128>" in ups[16], ups
    assert "conv_pipe" in ups[8], ups
    sub = _eps_with(net, x, t)
    assert torch.equal(sub, _eps_with(net, x, t))
    pipe = _eps_with(net, x, t, p4_sub=0)
    idx = [0, n // 2, n - 1]
    with torch.no_grad():
        ref = _oracle(a, synthetic_state_dict(a, 0))(xc[idx], tc[idx])
    d, e = _rel_l2(sub, pipe), _rel_l2(sub[idx], ref)
    print(f"n={n}: p4 sub-pixel vs conv_pipe rel-L2 {d:.2e}; vs oracle {e:.2e} (conv_pipe {_rel_l2(pipe[idx], ref):.2e})")
    assert d < 1e-2 and e < REL_L2_BF16


def test_p4_subpixel_convtranspose_vs_conv_pipe_cfg():
    """The CFG UpSample's ConvTranspose2d(5, 2, 2, 1) (ModelCondition.py:80) as 4 sub-pixel phases of 3x3
    taps on conv3x3_gn_p4_kernel (AB = 384: 16x16 -> 32x32 and 8x8 -> 16x16 inputs) against the same phase
    GEMMs on conv_pipe (p4_sub = 0) at C3's guided batch (2N = 64): within 1e-2 relative L2, deterministic,
    and the forward within the bf16 bound of the oracle."""
    a = ARCH_C
    net = _net(a, "bf16")
    n = 64
    gen = torch.Generator().manual_seed(640)
    xc = torch.randn(n, 3, 32, 32, generator=gen)
    tc = torch.randint(0, a.T, (n,), generator=gen)
    lab = torch.cat([torch.arange(n // 2) % 10 + 1, torch.zeros(n // 2, dtype=torch.long)])
    x, t, lb = xc.cuda(), tc.cuda(), lab.cuda()
    ops = net.native(n).profile_ops(x, t.to(torch.int32))
    convt = [o["kernel"] for o in ops if "384>" in o["kernel"]]
    assert any("conv3x3_gn_p4_kernel<16, 384>" in k for k in convt) and any("<8, 384>" in k for k in convt), convt

    def run(**opts):
        try:
            for k, v in opts.items():
                rt.set_option(k, v)
            return net(x, t, lb).float().cpu()
        finally:
            rt.set_option("p4_sub", 1)

    sub = run()
    assert torch.equal(sub, run())
    pipe = run(p4_sub=0)
    idx = [0, n - 1]
    with torch.no_grad():
        ref = _oracle(a, synthetic_state_dict(a, 0))(xc[idx], tc[idx], lab[idx])
    d, e = _rel_l2(sub, pipe), _rel_l2(sub[idx], ref)
    print(f"CFG 2N=64: p4 sub-pixel ConvTranspose vs conv_pipe rel-L2 {d:.2e}; vs oracle {e:.2e}")
    assert d < 1e-2 and e < REL_L2_BF16


def test_convtranspose_live_taps_vs_all_taps():
    """The CFG UpSample's ConvTranspose2d(5, 2, 2, 1) phases on conv3x3_gn_p4_kernel (8x8 -> 16x16 and
    16x16 -> 32x32 at 2N = 64) run only the taps of their 3x3 window that have a kernel tap (9 / 6 / 6 / 4:
    the others' weights are zero, pack_convt_subpix) and deal the phase tiles in cost-balanced pairs. A
    tile sums the same nonzero products in the same order, so the forward is bit-identical to the all-taps
    launch (convt_prune = 0), and within the bf16 bound of the oracle."""
    a = ARCH_C
    net = _net(a, "bf16")
    n = 64
    gen = torch.Generator().manual_seed(660)
    xc = torch.randn(n, 3, 32, 32, generator=gen)
    tc = torch.randint(0, a.T, (n,), generator=gen)
    lab = torch.cat([torch.arange(n // 2) % 10 + 1, torch.zeros(n // 2, dtype=torch.long)])
    x, t, lb = xc.cuda(), tc.cuda(), lab.cuda()
    ops = net.native(n).profile_ops(x, t.to(torch.int32))
    assert sum("384>" in o["kernel"] for o in ops) == 2, [o["kernel"] for o in ops]

    def run(prune):
        rt.set_option("convt_prune", prune)
        try:
            return net(x, t, lb).float().cpu()
        finally:
            rt.set_option("convt_prune", 1)

    live = run(1)
    assert torch.equal(live, run(0))
    idx = [0, n - 1]
    with torch.no_grad():
        ref = _oracle(a, synthetic_state_dict(a, 0))(xc[idx], tc[idx], lab[idx])
    e = _rel_l2(live[idx], ref)
    print(f"CFG 2N=64: live-tap ConvTranspose bit-identical to all taps; vs oracle {e:.2e}")
    assert e < REL_L2_BF16


@pytest.mark.parametrize("arch,n", [(ARCH_C, 64), (ARCH_A, 8)])
def test_subpixel_split_k_vs_unsplit(arch, n):
    """Under-filled sub-pixel conv_pipe launches (the CFG ConvTranspose2d from the 2x2 grid at 2N = 64:
    32 blocks; Arch A's 4x4 -> 8x8 upsample at n = 8: 16 blocks) split K over 4 phases x S slices with
    the in-launch combine (tickets per (phase, tile), slices summed in order): deterministic, within
    1e-2 relative L2 of the unsplit launch (subpix_split = 0), and within the bf16 bound of the oracle."""
    net = _net(arch, "bf16")
    gen = torch.Generator().manual_seed(650 + n)
    xc = torch.randn(n, 3, 32, 32, generator=gen)
    tc = torch.randint(0, arch.T, (n,), generator=gen)
    lab = torch.cat([torch.arange(n // 2) % 10 + 1, torch.zeros(n - n // 2, dtype=torch.long)]) if arch.cfg else None
    args = [xc.cuda(), tc.cuda()] + ([lab.cuda()] if arch.cfg else [])

    def run(split):
        rt.set_option("subpix_split", split)
        try:
            return net(*args).float().cpu()
        finally:
            rt.set_option("subpix_split", 1)

    sp = run(1)
    assert torch.equal(sp, run(1))
    un = run(0)
    idx = [0, n - 1]
    with torch.no_grad():
        ref = _oracle(arch, synthetic_state_dict(arch, 0))(xc[idx], tc[idx], *([lab[idx]] if arch.cfg else []))
    d, e = _rel_l2(sp, un), _rel_l2(sp[idx], ref)
    print(f"{arch.kind} n={n}: sub-pixel split-K vs unsplit rel-L2 {d:.2e}; vs oracle {e:.2e}")
    assert d < 1e-2 and e < REL_L2_BF16  # (measured 5.7e-3 / 7.8e-3: one conv's sum order, through the net)


def test_streaming_1x1_convs_vs_conv_pipe_n256():
    """The bench batch's ResBlock shortcuts at 32x32 / 16x16 / 8x8 (K = 128..640; K = 128 and 8x8 since round 6) on conv1x1_stream_kernel
    (weights resident in VGPRs, a 4-stage pixel-chunk ring across tiles): the same k order and
    the same MFMA as conv_pipe, so the forward is bit-identical to conv1x1 = 0; and vs the oracle."""
    a = ARCH_A
    net = _net(a, "bf16")
    n = 256
    gen = torch.Generator().manual_seed(670)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, a.T, (n,), generator=gen)
    ops = net.native(n).profile_ops(x.cuda(), t.to(torch.int32).cuda())
    k1 = [o for o in ops if "conv1x1_stream" in o["kernel"]]
    # (round 6: also the 8x8 level's shortcuts with K <= 640, 384 tiles on 240 persistent blocks)
    assert {o["H"] for o in k1} == {8, 16, 32}, [(o["H"], o["K"], o["kernel"]) for o in ops if o["ks"] == 1]

    def run(v):
        rt.set_option("conv1x1", v)
        try:
            return net(x.cuda(), t.cuda()).float().cpu()
        finally:
            rt.set_option("conv1x1", 1)

    st = run(1)
    assert torch.equal(st, run(0))
    idx = [0, 255]
    with torch.no_grad():
        ref = _oracle(a, synthetic_state_dict(a, 0))(x[idx], t[idx])
    assert _rel_l2(st[idx], ref) < REL_L2_BF16


def test_p4_96_cout_tiles_bit_identical_n256():
    """The 8x8 fused convs of the bench batch on 96-cout tiles (conv3x3_gn_p4_kernel<8, 512>: 256 tiles for the
    256 CUs instead of 192): every output's MFMA k order and every statistics slot's row order are the
    128-cout tiles', so the forward is bit-identical to p4_c96 = 0; and vs the oracle on images at both ends."""
    a = ARCH_A
    net = _net(a, "bf16")
    n = 256
    gen = torch.Generator().manual_seed(960)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, a.T, (n,), generator=gen)
    ops = net.native(n).profile_ops(x.cuda(), t.to(torch.int32).cuda())
    assert any("<8, 512>" in o["kernel"] for o in ops), sorted({o["kernel"] for o in ops})

    def run(v):
        rt.set_option("p4_c96", v)
        try:
            return net(x.cuda(), t.cuda()).float().cpu()
        finally:
            rt.set_option("p4_c96", 1)

    c96 = run(1)
    assert torch.equal(c96, run(1))
    assert torch.equal(c96, run(0))
    idx = [0, 255]
    with torch.no_grad():
        ref = _oracle(a, synthetic_state_dict(a, 0))(x[idx], t[idx])
    assert _rel_l2(c96[idx], ref) < REL_L2_BF16


@pytest.mark.parametrize("n", [16, 32])
def test_small_8x8_split_convs_vs_conv_pipe(n):
    """Small batches: the 8x8 level's plain convs whose 128x128 conv_pipe grid under-fills the chip run on
    conv_small's 64x64 whole-image tiles (option small_8x8), K split in-launch where a slice keeps >= 8 K-chunks
    (these K = 2304 convs run whole, the same k order as conv_pipe). Since
    round 5 the ResBlock shortcuts are folded into their block2 p5 conv, so at these batches the convs left on this
    path are the 16x16 -> 8x8 DownSample (3x3 s2) -- the census pins it, and that no 8x8 1x1 conv remains.
    Deterministic, within 1e-2 relative L2 of conv_pipe (small_8x8 = 0), bf16 bound vs oracle."""
    a = ARCH_A
    net = _net(a, "bf16")
    gen = torch.Generator().manual_seed(680 + n)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, a.T, (n,), generator=gen)
    ops = net.native(n).profile_ops(x.cuda(), t.to(torch.int32).cuda())
    small8 = [o for o in ops if o["kind"] == "conv" and o["H"] == 8 and "conv_small" in o["kernel"]]
    assert small8 and all(o["ks"] == 3 for o in small8), [(o["ks"], o["K"], o["kernel"]) for o in small8]
    assert not any(o["kind"] == "conv" and o["H"] == 8 and o["ks"] == 1 for o in ops)  # (shortcuts folded)

    def run(v):
        rt.set_option("small_8x8", v)
        try:
            return net(x.cuda(), t.cuda()).float().cpu()
        finally:
            rt.set_option("small_8x8", 1)

    w = run(1)
    assert torch.equal(w, run(1))
    p = run(0)
    idx = [0, n - 1]
    with torch.no_grad():
        ref = _oracle(a, synthetic_state_dict(a, 0))(x[idx], t[idx])
    d, e = _rel_l2(w, p), _rel_l2(w[idx], ref)
    print(f"n={n}: 8x8 conv_small vs conv_pipe rel-L2 {d:.2e}; vs oracle {e:.2e}")
    assert d < 1e-2 and e < REL_L2_BF16


@pytest.mark.parametrize("n", [16, 32])
def test_small_wide_stats_free_convs_vs_conv_pipe(n):
    """Small batches: the statistics-free 1x1 convs of 8x8 .. 32x32 images whose 128x128 conv_pipe grid
    under-fills the chip run on conv_small's 64x64 tiles (inside one image, split K; option small_wide). With the
    shortcut fold on (shipped) none is left at these batches -- the census pins that -- so the path is exercised
    with the fold off (p5_sc 0: the 15 ResBlock shortcuts, the form the fold's cost model falls back to where the
    extra slices cost more than the launch): deterministic, within 1e-2 relative L2 of conv_pipe (small_wide = 0)
    and within the bf16 bound of the oracle."""
    a = ARCH_A
    net = _net(a, "bf16")
    gen = torch.Generator().manual_seed(660 + n)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, a.T, (n,), generator=gen)
    ops = net.native(n).profile_ops(x.cuda(), t.to(torch.int32).cuda())
    assert not any(o["kind"] == "conv" and o["H"] >= 8 and o["ks"] == 1 for o in ops)  # (all folded)

    def run(v, census=False):
        rt.set_option("small_wide", v)
        rt.set_option("p5_sc", 0)
        try:
            o = net.native(n).profile_ops(x.cuda(), t.to(torch.int32).cuda()) if census else None
            return net(x.cuda(), t.cuda()).float().cpu(), o
        finally:
            rt.set_option("small_wide", 1)
            rt.set_option("p5_sc", 1)

    w, ops0 = run(1, census=True)
    wide = [o for o in ops0 if o["kind"] == "conv" and o["H"] >= 8 and o["ks"] == 1 and "conv_small" in o["kernel"]]
    assert len(wide) >= 5, [(o["H"], o["K"], o["kernel"]) for o in ops0 if o["ks"] == 1]  # (8 at n = 32: the 8x8 - 32x32 shortcuts)
    assert torch.equal(w, run(1)[0])
    p = run(0)[0]
    idx = [0, n - 1]
    with torch.no_grad():
        ref = _oracle(a, synthetic_state_dict(a, 0))(x[idx], t[idx])
    d, e = _rel_l2(w, p), _rel_l2(w[idx], ref)
    print(f"n={n}: conv_small (wide) vs conv_pipe rel-L2 {d:.2e}; vs oracle {e:.2e}")
    assert d < 1e-2 and e < REL_L2_BF16


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_dead_tap_pruning_archC_1x1_level(precision):
    """Arch C's 1x1 level (ModelCondition.py: ch_mult [1, 4, 8, 8, 4, 2] at 32 px): taps that read only padding for
    every output pixel are dropped at build time (option tap_prune) -- the 3x3 convs on 1x1 images run their centre
    tap (ks 1), the DownSample 2x2 -> 1x1 (c1 3x3 + c2 5x5, stride 2, merged into one 5x5 conv at build time, option
    down_merge) a 2x2 window, the ConvTranspose from the 1x1 grid its centre tap per phase. Exact in arithmetic (the
    dropped taps multiply zero padding): the census shows no 3x3+ conv left at H = 1 and exactly one merged
    DownSample, and a guided batch (2N = 64, the C3 leg's) matches the oracle (fp32 max|d| <= 2e-4, bf16 rel-L2
    <= 2e-2)."""
    a = ARCH_C
    net = _net(a, precision)
    n = 64
    gen = torch.Generator().manual_seed(641)
    xc = torch.randn(n, 3, 32, 32, generator=gen)
    tc = torch.randint(0, a.T, (n,), generator=gen)
    lab = torch.cat([torch.arange(n // 2) % 10 + 1, torch.zeros(n // 2, dtype=torch.long)])
    x, t, lb = xc.cuda(), tc.cuda(), lab.cuda()
    ops = net.native(n).profile_ops(x, t.to(torch.int32))
    h1 = [o for o in ops if o["kind"] == "conv" and o["H"] == 1]
    assert h1 and all(o["ks"] <= 2 for o in h1), [(o["ks"], o["K"], o["kernel"]) for o in h1]
    assert sum(o["ks"] == 2 for o in h1) == 1  # the DownSample into the 1x1 level (c1 + c2 as one 5x5 s2 conv)
    eps = net(x, t, lb).float().cpu()
    idx = [0, 31, 32, n - 1]
    with torch.no_grad():
        ref = _oracle(a, synthetic_state_dict(a, 0))(xc[idx], tc[idx], lab[idx])
    if precision == "fp32":
        d = (eps[idx] - ref).abs().max().item()
        print(f"Arch C 2N=64 fp32 (pruned taps) max|d| vs oracle {d:.2e}")
        assert d <= EPS_TOL_FP32
    else:
        e = _rel_l2(eps[idx], ref)
        print(f"Arch C 2N=64 bf16 (pruned taps, LDS-staged flash attention) rel-L2 vs oracle {e:.2e}")
        assert e < REL_L2_BF16


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-5), ("bf16", 1e-2)])
def test_one_token_attnblock_fold_archC(precision, tol):
    """Arch C's 1x1-level AttnBlocks (ModelCondition.py, one token): the softmax over a single key is exactly 1,
    so the block is x + proj(v(GN(x))); the build folds proj and v into one 1x1 conv (Wp Wv, Wp bv + bp in fp64)
    behind the GroupNorm (option attn_s1, read at create). Against the four-op path (attn_s1 = 0) on the same
    guided batch: relative L2 <= 1e-5 in fp32 (a reassociation of the two products), <= 1e-2 in bf16 (one bf16
    rounding of v fewer); and the folded forward against the oracle."""
    a = ARCH_C
    gen = torch.Generator().manual_seed(77)
    n = 8
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, a.T, (n,), generator=gen)
    lab = torch.arange(n) % 11
    outs = {}
    for v in (1, 0):
        rt.set_option("attn_s1", v)  # (read when the native UNet is built: at its first forward)
        try:
            net = _net(a, precision)
            outs[v] = net(x.cuda(), t.cuda(), lab.cuda()).float().cpu()
        finally:
            rt.set_option("attn_s1", 1)
        del net
        torch.cuda.empty_cache()
    assert not torch.equal(outs[1], outs[0])  # (the two builds differ: the fold took effect)
    d = _rel_l2(outs[1], outs[0])
    with torch.no_grad():
        ref = _oracle(a, synthetic_state_dict(a, 0))(x[:2], t[:2], lab[:2])
    e = _rel_l2(outs[1][:2], ref)
    print(f"Arch C {precision}: folded one-token AttnBlocks vs four-op path rel-L2 {d:.2e}; vs oracle {e:.2e}")
    assert d <= tol
    assert e <= (1e-4 if precision == "fp32" else REL_L2_BF16)


def test_forward_bf16_full_batch_vs_oracle_subset():
    """The bench batch (N=256) runs the persistent fused convs with several tiles per block
    (4 at 32x32, 2 at 16x16), the 2-blocks-per-image attention grid and the split-K small level: images
    spread over the batch match the oracle (fp32, CPU) within the bf16 bound."""
    a = ARCH_A
    net = _net(a, "bf16")
    n = 256
    gen = torch.Generator().manual_seed(256)
    x = torch.randn(n, 3, 32, 32, generator=gen)
    t = torch.randint(0, 1000, (n,), generator=gen)
    eps = net(x.cuda(), t.cuda()).float().cpu()
    idx = torch.tensor([0, 1, 63, 128, 200, 255])
    with torch.no_grad():
        ref = _oracle(a, synthetic_state_dict(a, 0))(x[idx], t[idx])
    for k, i in enumerate(idx.tolist()):
        assert _rel_l2(eps[i], ref[k]) < REL_L2_BF16, (i, _rel_l2(eps[i], ref[k]))


# ----------------------------------------------------------------------------- surface / forced fallbacks
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_cfg_return_representation_vs_oracle(precision):
    """``UNet.forward(x, t, labels, return_representation=True)`` (ModelCondition.py:206,225-235):
    (eps, h) with h the pre-tail activation as NCHW fp32, against the oracle's pre-tail tensor
    (fp32: max|d| <= 2e-4 on the tiny CFG UNet; bf16: rel-L2 <= 2e-2 on Arch C)."""
    a = ARCH_TINY_CFG if precision == "fp32" else ARCH_C
    sd = synthetic_state_dict(a, 0)
    net = _net(a, precision)
    gen = torch.Generator().manual_seed(17)
    x = torch.randn(3, 3, 32, 32, generator=gen)
    t = torch.randint(0, a.T, (3,), generator=gen)
    lab = torch.tensor([0, 4, 10])
    eps, rep = net(x.cuda(), t.cuda(), lab.cuda(), return_representation=True)
    e_only = net(x.cuda(), t.cuda(), lab.cuda())
    assert torch.equal(eps, e_only)
    with torch.no_grad():
        r_eps, r_rep = R.unet_forward(sd, x, t, a.ch, a.ch_mult, a.attn, a.num_res_blocks, labels=lab, cfg=True,
                                      return_representation=True)
    assert tuple(rep.shape) == tuple(r_rep.shape) == (3, a.ch * a.ch_mult[0], 32, 32)
    if precision == "fp32":
        np.testing.assert_allclose(rep.cpu().numpy(), r_rep.numpy(), atol=EPS_TOL_FP32, rtol=0)
    else:
        e = _rel_l2(rep.cpu(), r_rep)
        print(f"Arch C bf16 pre-tail representation rel-L2 {e:.3e}")
        assert e < REL_L2_BF16


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_forced_register_staged_conv_vs_reference(precision):
    """conv_igemm (the register-staged implicit-GEMM conv that conv_variant = 1 forces for every plain
    conv: 1x1 shortcuts, q|k|v / proj, 3x3 stride-2 downsamples) on Arch A: fp32 against the
    reference's own eps (archA_eps.npz, max|d| <= 2e-4), bf16 against the oracle (rel-L2 <= 2e-2).
    (The other fallback-looking kernels -- head_kernel, tail2_kernel / tail_kernel, attn_kernel -- are
    the fp32 parity path and run in every fp32 test above.)"""
    g = golden("archA_eps")
    x, t = torch.from_numpy(g["x"]), torch.from_numpy(g["t"])
    rt.set_option("conv_variant", 1)
    try:
        net = _net(ARCH_A, precision)
        eps = net(x.cuda(), t.cuda()).cpu()
    finally:
        rt.set_option("conv_variant", 2)
    if precision == "fp32":
        np.testing.assert_allclose(eps.numpy(), g["eps"], atol=EPS_TOL_FP32, rtol=0)
    else:
        assert _rel_l2(eps, torch.from_numpy(g["eps"])) < REL_L2_BF16
