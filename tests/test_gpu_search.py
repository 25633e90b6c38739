"""GPU parity of the headline bf16 path, the search products, the extended-T / full-T
configs and the sampler's run-time behaviour -- all through the C ABI.

Tolerances ("Parity"):
  bf16 Arch A trajectory x0, T = 20, injected reference noise   rel-L2 <= 3e-2
  fp32 sampler windows vs the oracle (20 steps)                 max|d| <= 2e-3
  fp32 vs bf16 search round (same Philox noise, T = 1000)       argmax identical whenever the fp32
                                                                top-2 gap > 1e-3; per-candidate
                                                                |score_bf16 - score_fp32| <= 2e-3
  search products vs search_T5.npz (reference run)              scores <= 1e-5, argmax / best noise exact
"""
import dataclasses
import math
import os

import numpy as np
import pytest
import torch
import yaml

from conftest import golden
from oracle import ref_cpu as R
from itsd import entry as E
from itsd import runtime as rt
from itsd.arch import ARCH_A, ARCH_TINY, ARCH_TINY_CFG
from itsd.diffusion import GaussianDiffusionSampler, reference_noise_plan
from itsd.model import CondUNet, UNet
from itsd.search import PathSearch, RandomSearch, SearchEngine, ZeroOrderSearch
from itsd.verifier import OracleVerifier
from itsd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

TRAJ_TOL_FP32 = 2e-3
REL_L2_BF16_TRAJ = 3e-2


def _net(a, precision="fp32", seed=0):
    if a.cfg:
        net = CondUNet(a.T, a.num_labels, a.ch, a.ch_mult, a.num_res_blocks, 0.0, img_size=a.img_size,
                       precision=precision)
    else:
        net = UNet(a.T, a.ch, a.ch_mult, a.attn, a.num_res_blocks, 0.0, img_size=a.img_size, precision=precision)
    net.load_state_dict(synthetic_state_dict(a, seed))
    return net.to("cuda:0")


def _rel_l2(a, b):
    return (torch.linalg.norm((a - b).flatten()) / torch.linalg.norm(b.flatten())).item()


def _oracle_fw(a, seed=0):
    sd = synthetic_state_dict(a, seed)
    return lambda x, t: R.unet_forward(sd, x, t, a.ch, a.ch_mult, a.attn, a.num_res_blocks)


# ----------------------------------------------------------------------------- headline bf16 path
def test_trajectory_archA_bf16_vs_reference():
    """The bench's arch and precision (Arch A, bf16) over the reference's own T = 20
    trajectory (archA_traj.npz) with the reference's noise injected."""
    g = golden("archA_traj")
    T = int(g["T"])
    torch.manual_seed(int(g["seed"]))
    x_T, noise = reference_noise_plan((2, 3, 32, 32), T, n_runs=1)
    smp = GaussianDiffusionSampler(_net(ARCH_A, "bf16"), 1e-4, 0.02, T)
    x0 = smp(x_T[0].cuda(), noise=noise).cpu()
    err = _rel_l2(x0, torch.from_numpy(g["x0"]))
    print(f"bf16 Arch A T=20 trajectory rel-L2 vs reference: {err:.3e}")
    assert err <= REL_L2_BF16_TRAJ


def test_fp32_bf16_search_argmax_agreement():
    """one Philox random-search round of 32 candidates at T = 1000 on Arch A in
    fp32 and in bf16 (identical x_T and per-step noise): the argmax agrees whenever the
    fp32 top-2 gap exceeds 1e-3, and every candidate's score stays within 2e-3 (measured 3.1e-4)."""
    scores = {}
    for prec in ("fp32", "bf16"):
        smp = GaussianDiffusionSampler(_net(ARCH_A, prec), 1e-4, 0.02, 1000)
        eng = SearchEngine(smp, OracleVerifier(), seed=11)
        _, _, info = eng.random_search(32, (1, 3, 32, 32))
        scores[prec] = torch.tensor(info["scores"], dtype=torch.float64)
        del smp, eng
        torch.cuda.empty_cache()
    f, b = scores["fp32"], scores["bf16"]
    assert torch.isfinite(f).all() and torch.isfinite(b).all()
    top2 = torch.topk(f, 2).values
    gap = (top2[0] - top2[1]).item()
    d = (f - b).abs().max().item()
    print(f"fp32 vs bf16 scores: max|d| = {d:.3e}, fp32 top-2 gap = {gap:.3e}, "
          f"argmax fp32 {int(torch.argmax(f))} bf16 {int(torch.argmax(b))}")
    if gap > 1e-3:
        assert int(torch.argmax(f)) == int(torch.argmax(b))
    assert d <= 2e-3


# ----------------------------------------------------------------------------- search products
def test_product_searches_sequential_vs_reference_T5():
    """RandomSearch / ZeroOrderSearch / PathSearch.search (the product classes, sequential
    API) with the native sampler's denoise_fn consuming the reference's per-step draws and
    the native OracleVerifier: scores, best score and best noise of search_T5.npz."""
    g = golden("search_T5")
    smp = GaussianDiffusionSampler(_net(ARCH_TINY), 1e-4, 0.02, 5)
    dn, ver = smp.denoise_fn(reference_rng=True), OracleVerifier()
    rec = []

    def vf(images, **kw):
        s = ver(images)
        rec.append(s)
        return s

    shape = (1, 3, 32, 32)
    torch.manual_seed(0)
    rs = RandomSearch(n_candidates=4)
    bn, bs = rs.search(shape, dn, vf, device="cpu", verbose=False)
    np.testing.assert_allclose(rec, g["random_scores"], atol=1e-5)
    np.testing.assert_array_equal(bn.numpy(), g["random_best_noise"])
    assert rs.nfes == int(g["random_nfes"])
    rec.clear()
    torch.manual_seed(1)
    init = torch.randn(shape)
    zo = ZeroOrderSearch(n_neighbors=3, lambda_radius=0.95, n_iterations=2)
    bn, bs, h = zo.search(init, dn, vf, device="cpu", verbose=False)
    np.testing.assert_allclose(np.array(h["scores"]), g["zo_scores"], atol=1e-5)
    np.testing.assert_array_equal(bn.numpy(), g["zo_best_noise"])
    assert abs(bs - float(g["zo_best_score"])) < 1e-5 and zo.nfes == int(g["zo_nfes"])
    rec.clear()
    torch.manual_seed(2)
    init = torch.randn(shape)
    ps = PathSearch(n_paths=3, injection_step=400, noise_scale=0.1)
    bn, bs, h = ps.search(init, dn, vf, timesteps=5, device="cpu", verbose=False)
    np.testing.assert_allclose(np.array(h["scores"]), g["path_scores"], atol=1e-5)
    np.testing.assert_array_equal(bn.numpy(), g["path_best_noise"])
    assert ps.nfes == int(g["path_nfes"])


def test_product_searches_batched_reference_mode_vs_reference_T5():
    """The same three searches through the batched engine (one native sampler run per round)
    in parity mode (reference draw order): scores, argmax, best noise of search_T5.npz."""
    g = golden("search_T5")
    smp = GaussianDiffusionSampler(_net(ARCH_TINY), 1e-4, 0.02, 5)
    ver = OracleVerifier()
    shape = (1, 3, 32, 32)
    torch.manual_seed(0)
    rs = RandomSearch(n_candidates=4)
    bn, bs = rs.search(shape, None, ver, batched=True, sampler=smp, reference_rng=True)
    np.testing.assert_array_equal(bn.cpu().numpy(), g["random_best_noise"])
    assert abs(bs - float(g["random_best_score"])) < 1e-5
    torch.manual_seed(1)
    init = torch.randn(shape)
    zo = ZeroOrderSearch(n_neighbors=3, lambda_radius=0.95, n_iterations=2)
    bn, bs, h = zo.search(init, None, ver, batched=True, sampler=smp, reference_rng=True)
    np.testing.assert_allclose(np.array(h["scores"]), g["zo_scores"], atol=1e-5)
    np.testing.assert_array_equal(bn.cpu().numpy(), g["zo_best_noise"])
    assert abs(bs - float(g["zo_best_score"])) < 1e-5 and zo.nfes == int(g["zo_nfes"])
    torch.manual_seed(2)
    init = torch.randn(shape)
    ps = PathSearch(n_paths=3, injection_step=400, noise_scale=0.1)
    bn, bs, h = ps.search(init, None, ver, batched=True, sampler=smp, reference_rng=True)
    np.testing.assert_allclose(np.array(h["scores"]), g["path_scores"], atol=1e-5)
    np.testing.assert_array_equal(bn.cpu().numpy(), g["path_best_noise"])


def test_best_image_is_the_scored_trajectory():
    """the search's best image is the denoised candidate that earned best_score
    (rescoring it reproduces the score), for the Philox engine's random and zero-order search."""
    smp = GaussianDiffusionSampler(_net(ARCH_TINY, "bf16"), 1e-4, 0.02, 50)
    ver = OracleVerifier()
    eng = SearchEngine(smp, ver, seed=4)
    _, score, _ = eng.random_search(8, (1, 3, 32, 32))
    assert abs(ver.score(eng.best_image) - score) < 1e-9
    _, score, _ = eng.zero_order_search(eng.initial_noise((1, 3, 32, 32)), 4, 0.95, 3)
    assert abs(ver.score(eng.best_image) - score) < 1e-9


# ----------------------------------------------------------------------------- sampler run-time behaviour
def test_graph_captured_once_across_zero_order_rounds():
    """The step graph is keyed by (batch, buffers, options); seed / noise offset / clip step are
    device-side run parameters, so a 3-round zero-order search captures ONE graph -- and its
    results equal the eager (no-graph) run bit for bit."""
    net = _net(ARCH_TINY, "bf16")
    smp = GaussianDiffusionSampler(net, 1e-4, 0.02, 20)
    res = {}
    for graph in (True, False):
        eng = SearchEngine(smp, OracleVerifier(), seed=2, graph=graph)
        nat = net.native(8)
        before = nat.query("graph_captures")
        init = eng.initial_noise((1, 3, 32, 32))
        bn, bs, h = eng.zero_order_search(init, 8, 0.95, 3)
        res[graph] = (bn.cpu(), bs, h["scores"], nat.query("graph_captures") - before)
    assert res[True][3] == 1 and res[False][3] == 0
    assert torch.equal(res[True][0], res[False][0]) and res[True][1] == res[False][1]
    assert res[True][2] == res[False][2]


def test_nan_in_noise_raises_assertion():
    """Diffusion.py:100 `assert torch.isnan(x_t).int().sum() == 0, "nan in tensor."`: the
    device NaN flag is raised by the tail kernel and reported once at the end of the run."""
    smp = GaussianDiffusionSampler(_net(ARCH_TINY), 1e-4, 0.02, 4)
    x = torch.randn(2, 3, 32, 32)
    noise = torch.randn(4, 2, 3, 32, 32)
    noise[2, 1, 0, 5, 7] = float("nan")
    for graph in (True, False):
        with pytest.raises(AssertionError, match="nan in tensor"):
            smp(x.cuda(), noise=noise, graph=graph)
    out = smp(x.cuda(), noise=torch.randn(4, 2, 3, 32, 32))  # the flag is reset per run
    assert torch.isfinite(out).all()


def test_philox_noise_kernel_matches_oracle():
    """itsd_noise (candidate x_T) == the numpy Philox restatement, element for element."""
    out = torch.empty(3, 3, 32, 32, device="cuda")
    rt.noise(out, 3, seed=77, stream_id=0xF0000005, cand_offset=2)
    ref = R.philox_normal(77, 0xF0000005, np.arange(2 * 3072, 5 * 3072)).reshape(3, 3, 32, 32)
    np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), atol=2e-6, rtol=2e-6)


def _philox_window(a, T, t_begin, steps, n, seed, offset_cands=0, bT=0.02):
    """Run the product sampler in Philox mode for `steps` steps from t_begin and the oracle
    loop with the same counter-based noise; return both."""
    net = _net(a)
    smp = GaussianDiffusionSampler(net, 1e-4, bT, T)
    gen = torch.Generator().manual_seed(T + n)
    x = torch.randn(n, 3, a.img_size, a.img_size, generator=gen)
    per = 3 * a.img_size * a.img_size
    t_end = t_begin - steps + 1
    got = smp.run(x.cuda().contiguous(), t_begin=t_begin, t_end=t_end, seed=seed, noise_offset=offset_cands * per).cpu()
    s = R.schedule(1e-4, bT, T)
    base = offset_cands * per

    def nf(step, xx):
        return R.philox_normal(seed, step, np.arange(base, base + xx.numel())).reshape(xx.shape)

    with torch.no_grad():
        ref = R.p_sample_loop(_oracle_fw(a), x, s, nf, t_begin=t_begin, t_end=t_end, clip=t_end == 0)
    return got, ref


def test_C1_archA_T1000_philox_window_fp32_vs_oracle():
    """C1 (Main.py eval, Arch A, T = 1000, N = 1): the first 20 ancestral steps t = 999..980 of
    the product's Philox-mode sampler against the oracle fed the same counter-based noise."""
    got, ref = _philox_window(ARCH_A, 1000, 999, 20, 1, seed=123)
    np.testing.assert_allclose(got.numpy(), ref.numpy(), atol=TRAJ_TOL_FP32, rtol=0)


def test_C5_extended_T3000_window_fp32_vs_oracle():
    """C5 schedule (fine_tune_extended_T.py: T = 3000, linspace(1e-4, 0.02, 3000)): itsd_set_schedule
    with T = 3000 (a 3000 x 7424 temb table) and the steps t = 2999..2980 against the oracle."""
    got, ref = _philox_window(ARCH_A, 3000, 2999, 20, 2, seed=9, offset_cands=5)
    np.testing.assert_allclose(got.numpy(), ref.numpy(), atol=TRAJ_TOL_FP32, rtol=0)


def test_C5_path_search_round_T3000_bf16():
    """C5's algorithm at its T: one bf16 PathSearch round (search_algorithm.py:265-336) of 8
    paths over the full 3000 steps -- finite, clipped, strict-'>' argmax, scored image kept."""
    smp = GaussianDiffusionSampler(_net(ARCH_A, "bf16"), 1e-4, 0.02, 3000)
    eng = SearchEngine(smp, OracleVerifier(), seed=5)
    init = eng.initial_noise((1, 3, 32, 32))
    best, score, h = eng.path_search(init, 8, 0.1, 400)
    sc = torch.tensor(h["scores"], dtype=torch.float64)
    assert torch.isfinite(sc).all() and score == sc.max().item() and h["best_index"] == int(torch.argmax(sc))
    assert eng.best_image.abs().max().item() <= 1.0
    assert torch.equal(best, eng.candidate_noise(0, h["best_index"], 1, (1, 3, 32, 32), pivot=init, scale=0.1))


def test_C1_main_eval_archA_T1000_batch1(tmp_path):
    """C1 end to end: Main.py's eval (config.yaml keys) on Arch A, inference_T = 1000,
    batch_size = 1, synthetic weights, fp32: equals a hand-run of the same sampler."""
    cfg = E.load_config(None, ["weights=random", "batch_size=1", "inference_T=1000", f"sampled_dir={tmp_path}",
                               "seed=7", "nrow=1"])
    res = E.run(cfg)
    torch.manual_seed(7)
    net = UNet(1000, 128, [1, 2, 3, 4], [2], 2, 0.0, weights="gauss").to("cuda:0")
    x = torch.randn(1, 3, 32, 32, device="cuda:0")
    assert torch.equal(x, res["noisy"])
    ref = GaussianDiffusionSampler(net, 1e-4, 0.02, 1000)(x) * 0.5 + 0.5
    assert torch.equal(ref, res["sampled"])
    assert os.path.exists(os.path.join(tmp_path, cfg["sampledImgName"]))


# ----------------------------------------------------------------------------- inference_config surface
_REF_KEYS = ("checkpoint_path", "T", "beta_1", "beta_T", "img_size", "time_embedding_strategy",
             "fine_tune_time_embedding", "channel", "channel_mult", "attn", "num_res_blocks", "dropout", "device",
             "use_multi_gpu", "device_ids", "batch_size", "metric_interval", "imagenet_root", "use_val_for_eval",
             "fid_num_real_samples", "clip_num_real_samples", "output_dir", "metrics_save_dir",
             "sampled_images_save_dir", "nrow")


def test_inference_config_reference_keys_end_to_end(tmp_path):
    """A YAML holding exactly the reference's inference_config.yaml keys (Arch A checkpoint,
    T = 3000 -- where the reference misdetects T = 512 and breaks its own Linear) runs through
    entry.load_config + run: a PNG in sampled_images_save_dir and metrics_history.json in
    output_dir, images equal to a hand-run sampler with the checkpoint's weights."""
    sd = synthetic_state_dict(ARCH_A, 8)
    ck = tmp_path / "ep15_bs40_T1000_lr1e-4" / "ckpt_0_.pt"
    ck.parent.mkdir()
    torch.save({"module." + k: v for k, v in sd.items()}, str(ck))
    vals = dict(checkpoint_path=str(ck), T=3000, beta_1=1e-4, beta_T=0.02, img_size=32,
                time_embedding_strategy="interpolate", fine_tune_time_embedding=False, channel=128,
                channel_mult=[1, 2, 3, 4], attn=[2], num_res_blocks=2, dropout=0.15, device="cuda",
                use_multi_gpu=True, device_ids=[0], batch_size=2, metric_interval=30, imagenet_root="/none",
                use_val_for_eval=True, fid_num_real_samples=5000, clip_num_real_samples=5000,
                output_dir=str(tmp_path / "out"), metrics_save_dir=str(tmp_path / "curves"),
                sampled_images_save_dir=str(tmp_path / "imgs"), nrow=8)
    assert set(vals) == set(_REF_KEYS)
    p = tmp_path / "inference_config.yaml"
    p.write_text(yaml.safe_dump(vals))
    cfg = E.load_config(str(p), ["seed=3"])
    res = E.run(cfg)
    pngs = os.listdir(tmp_path / "imgs")
    assert len(pngs) == 1 and pngs[0].startswith("ep15_bs40_T1000_lr1e-4_T3000_bs2_size32_")
    assert os.path.exists(tmp_path / "out" / "metrics_history.json")
    torch.manual_seed(3)
    net = UNet(3000, 128, [1, 2, 3, 4], [2], 2, 0.0).to("cuda:0")
    net.load_state_dict(sd)
    x = torch.randn(2, 3, 32, 32, device="cuda:0")
    ref = GaussianDiffusionSampler(net, 1e-4, 0.02, 3000)(x) * 0.5 + 0.5
    assert torch.equal(ref, res["sampled"])


def test_cfg_checkpoint_T_mismatch_interpolate(tmp_path):
    """MainCondition eval with a table time embedding of 600 rows and T = 900: strategy
    'interpolate' rebuilds the table (abstract_metrics...:211-248) and samples; without a
    strategy the mismatch raises."""
    a_ck = dataclasses.replace(ARCH_TINY_CFG, T=600)
    sd = synthetic_state_dict(a_ck, 6)
    torch.save(sd, str(tmp_path / "ckpt.pt"))
    base = [f"save_dir={tmp_path}", "test_load_weight=ckpt.pt", "T=900", "channel=32", "channel_mult=[1,2]",
            "num_res_blocks=1", "batch_size=10", f"sampled_dir={tmp_path}", "seed=1"]
    with pytest.raises(ValueError):
        E.run(E.load_config(None, base, config_name="condition_config"), condition=True)
    res = E.run(E.load_config(None, base + ["time_embedding_strategy=interpolate"], config_name="condition_config"),
                condition=True)
    assert torch.isfinite(res["sampled"]).all() and res["sampled"].shape == (10, 3, 32, 32)


# ----------------------------------------------------------------------------- 256 px
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_forward_256px_vs_reference(precision):
    """Arch A at 256 px (the reference's ImageNet runs and inference_config img_size):
    fp32 max-abs 2e-4, bf16 rel-L2 2e-2 against the reference's own eps (archA256_eps.npz)."""
    g = golden("archA256_eps")
    a = dataclasses.replace(ARCH_A, img_size=256)
    eps = _net(a, precision)(torch.from_numpy(g["x"]).cuda(), torch.from_numpy(g["t"]).cuda()).cpu()
    ref = torch.from_numpy(g["eps"])
    if precision == "fp32":
        np.testing.assert_allclose(eps.numpy(), ref.numpy(), atol=2e-4, rtol=0)
    else:
        assert _rel_l2(eps, ref) < 2e-2
