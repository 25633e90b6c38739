"""ORACLE (test infrastructure only; never imported by the product package).

Functional PyTorch-CPU fp32 restatement of the reference hot path, driven by a
plain state_dict. Every function cites the reference lines it restates.
Pinned against reference outputs in ``tests/golden`` (see oracle/__init__.py).
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
SD = Dict[str, Tensor]


# --------------------------------------------------------------------------- schedule
def schedule(beta_1: float, beta_T: float, T: int) -> Dict[str, Tensor]:
    """``Diffusion/Diffusion.py:57-65`` and the var of ``:76``."""
    betas = torch.linspace(beta_1, beta_T, T).double()
    alphas = 1.0 - betas
    ab = torch.cumprod(alphas, dim=0)
    ab_prev = F.pad(ab, [1, 0], value=1)[:T]
    c1 = torch.sqrt(1.0 / alphas)
    c2 = c1 * (1.0 - alphas) / torch.sqrt(1.0 - ab)
    pv = betas * (1.0 - ab_prev) / (1.0 - ab)
    var = torch.cat([pv[1:2], betas[1:]])
    return {"betas": betas, "coeff1": c1, "coeff2": c2, "posterior_var": pv, "var": var}


def _extract(v: Tensor, t: Tensor, ndim: int) -> Tensor:
    """``Diffusion.py:9-16``: gather then cast to fp32, shaped [B,1,1,1]."""
    out = torch.gather(v, index=t, dim=0).float()
    return out.view([t.shape[0]] + [1] * (ndim - 1))


# --------------------------------------------------------------------------- UNet
def _silu(x: Tensor) -> Tensor:
    return x * torch.sigmoid(x)  # Swish, Model.py:10-12


def _layout(ch: int, ch_mult: Sequence[int], attn: Sequence[int], nrb: int, cfg: bool):
    """Module-list layout of ``Model.py:218-246`` / ``ModelCondition.py:171-197``:
    returns (down, mid, up) lists of (prefix, kind, in_ch, out_ch, attn)."""
    down, up = [], []
    chs, now = [ch], ch
    for i, m in enumerate(ch_mult):
        out = ch * m
        for _ in range(nrb):
            down.append((f"downblocks.{len(down)}", "res", now, out, True if cfg else (i in attn)))
            now = out
            chs.append(now)
        if i != len(ch_mult) - 1:
            down.append((f"downblocks.{len(down)}", "down", now, now, False))
            chs.append(now)
    mid = [("middleblocks.0", "res", now, now, True), ("middleblocks.1", "res", now, now, False)]
    for i, m in reversed(list(enumerate(ch_mult))):
        out = ch * m
        for _ in range(nrb + 1):
            up.append((f"upblocks.{len(up)}", "res", chs.pop() + now, out, False if cfg else (i in attn)))
            now = out
        if i != 0:
            up.append((f"upblocks.{len(up)}", "up", now, now, False))
    return down, mid, up


def attn_block(sd: SD, p: str, x: Tensor) -> Tensor:
    """``Model.py:145-164`` (CFG twin ``ModelCondition.py:98-117``)."""
    B, C, H, W = x.shape
    h = F.group_norm(x, 32, sd[p + ".group_norm.weight"], sd[p + ".group_norm.bias"], 1e-5)
    q = F.conv2d(h, sd[p + ".proj_q.weight"], sd[p + ".proj_q.bias"])
    k = F.conv2d(h, sd[p + ".proj_k.weight"], sd[p + ".proj_k.bias"])
    v = F.conv2d(h, sd[p + ".proj_v.weight"], sd[p + ".proj_v.bias"])
    q = q.permute(0, 2, 3, 1).reshape(B, H * W, C)
    k = k.reshape(B, C, H * W)
    w = torch.bmm(q, k) * (int(C) ** (-0.5))
    w = F.softmax(w, dim=-1)
    v = v.permute(0, 2, 3, 1).reshape(B, H * W, C)
    h = torch.bmm(w, v)
    h = h.view(B, H, W, C).permute(0, 3, 1, 2)
    h = F.conv2d(h, sd[p + ".proj.weight"], sd[p + ".proj.bias"])
    return x + h


def res_block(sd: SD, p: str, x: Tensor, temb: Tensor, in_ch: int, out_ch: int, use_attn: bool,
              cemb: Optional[Tensor] = None) -> Tensor:
    """``Model.py:202-209`` (CFG ``ModelCondition.py:153-161`` adds cond_proj)."""
    h = F.group_norm(x, 32, sd[p + ".block1.0.weight"], sd[p + ".block1.0.bias"], 1e-5)
    h = F.conv2d(_silu(h), sd[p + ".block1.2.weight"], sd[p + ".block1.2.bias"], padding=1)
    h = h + F.linear(_silu(temb), sd[p + ".temb_proj.1.weight"], sd[p + ".temb_proj.1.bias"])[:, :, None, None]
    if cemb is not None:
        h = h + F.linear(_silu(cemb), sd[p + ".cond_proj.1.weight"], sd[p + ".cond_proj.1.bias"])[:, :, None, None]
    h = F.group_norm(h, 32, sd[p + ".block2.0.weight"], sd[p + ".block2.0.bias"], 1e-5)
    h = F.conv2d(_silu(h), sd[p + ".block2.3.weight"], sd[p + ".block2.3.bias"], padding=1)
    if in_ch != out_ch:
        h = h + F.conv2d(x, sd[p + ".shortcut.weight"], sd[p + ".shortcut.bias"])
    else:
        h = h + x
    if use_attn:
        h = attn_block(sd, p + ".attn", h)
    return h


def time_embedding(sd: SD, t: Tensor, d_model: int) -> Tensor:
    """Functional sinusoid + MLP, ``Model.py:51-93``."""
    B = t.shape[0]
    e = t.float().unsqueeze(-1) * sd["time_embedding.freq_coeffs"].unsqueeze(0)
    e = torch.stack([torch.sin(e), torch.cos(e)], dim=-1).reshape(B, d_model)
    h = F.linear(e, sd["time_embedding.timembedding.0.weight"], sd["time_embedding.timembedding.0.bias"])
    return F.linear(_silu(h), sd["time_embedding.timembedding.2.weight"], sd["time_embedding.timembedding.2.bias"])


def _mlp_from_table(sd: SD, p: str, idx: Tensor) -> Tensor:
    """Embedding -> Linear -> Swish -> Linear (``ModelCondition.py:37-46,53-62``)."""
    e = F.embedding(idx, sd[p + ".0.weight"])
    h = F.linear(e, sd[p + ".1.weight"], sd[p + ".1.bias"])
    return F.linear(_silu(h), sd[p + ".3.weight"], sd[p + ".3.bias"])


def unet_forward(sd: SD, x: Tensor, t: Tensor, ch: int, ch_mult: Sequence[int], attn: Sequence[int],
                 num_res_blocks: int, labels: Optional[Tensor] = None, cfg: bool = False,
                 return_representation: bool = False):
    """``Model.py:265-285`` (DDPM) / ``ModelCondition.py:206-235`` (CFG; with
    ``return_representation`` it returns (eps, h) with h the pre-tail activation, ``:225-235``)."""
    if cfg:
        temb = _mlp_from_table(sd, "time_embedding.timembedding", t)
        cemb = _mlp_from_table(sd, "cond_embedding.condEmbedding", labels)
    else:
        temb = time_embedding(sd, t, ch)
        cemb = None
    down, mid, up = _layout(ch, ch_mult, attn, num_res_blocks, cfg)
    h = F.conv2d(x, sd["head.weight"], sd["head.bias"], padding=1)
    hs = [h]
    for (p, kind, cin, cout, a) in down:
        if kind == "res":
            h = res_block(sd, p, h, temb, cin, cout, a, cemb)
        elif cfg:  # DownSample ModelCondition.py:71-73
            h = (F.conv2d(h, sd[p + ".c1.weight"], sd[p + ".c1.bias"], stride=2, padding=1)
                 + F.conv2d(h, sd[p + ".c2.weight"], sd[p + ".c2.bias"], stride=2, padding=2))
        else:  # DownSample Model.py:106-108
            h = F.conv2d(h, sd[p + ".main.weight"], sd[p + ".main.bias"], stride=2, padding=1)
        hs.append(h)
    for (p, kind, cin, cout, a) in mid:
        h = res_block(sd, p, h, temb, cin, cout, a, cemb)
    for (p, kind, cin, cout, a) in up:
        if kind == "res":
            h = torch.cat([h, hs.pop()], dim=1)  # Model.py:279-280
            h = res_block(sd, p, h, temb, cin, cout, a, cemb)
        elif cfg:  # UpSample ModelCondition.py:82-86
            h = F.conv_transpose2d(h, sd[p + ".t.weight"], sd[p + ".t.bias"], stride=2, padding=2,
                                   output_padding=1)
            h = F.conv2d(h, sd[p + ".c.weight"], sd[p + ".c.bias"], padding=1)
        else:  # UpSample Model.py:121-126
            h = F.interpolate(h, scale_factor=2, mode="nearest")
            h = F.conv2d(h, sd[p + ".main.weight"], sd[p + ".main.bias"], padding=1)
    rep = h  # ModelCondition.py:225 last_representation
    h = F.group_norm(h, 32, sd["tail.0.weight"], sd["tail.0.bias"], 1e-5)
    h = F.conv2d(_silu(h), sd["tail.2.weight"], sd["tail.2.bias"], padding=1)
    assert not hs
    return (h, rep) if return_representation else h


# --------------------------------------------------------------------------- sampler
def p_sample_loop(model_fn: Callable[[Tensor, Tensor], Tensor], x_T: Tensor, sched: Dict[str, Tensor],
                  noise_fn: Callable[[int, Tensor], Tensor], t_begin: Optional[int] = None,
                  t_end: int = 0, clip: bool = True) -> Tensor:
    """Ancestral sampler ``Diffusion.py:84-102`` (CFG ``DiffusionCondition.py:89-105``
    with ``model_fn`` returning the guided eps). ``noise_fn(step, x_t)`` supplies the
    ``randn_like`` draw of ``:96`` (called for step > 0 only, in loop order)."""
    T = sched["coeff1"].shape[0]
    t_begin = T - 1 if t_begin is None else t_begin
    x = x_T
    for step in range(t_begin, t_end - 1, -1):
        t = torch.full((x.shape[0],), step, dtype=torch.long)
        var = _extract(sched["var"], t, x.ndim)
        eps = model_fn(x, t)
        mean = _extract(sched["coeff1"], t, x.ndim) * x - _extract(sched["coeff2"], t, x.ndim) * eps
        noise = noise_fn(step, x) if step > 0 else 0
        x = mean + torch.sqrt(var) * noise
        assert torch.isnan(x).int().sum() == 0, "nan in tensor."
    return torch.clip(x, -1, 1) if clip else x


def cfg_eps(model_fn3: Callable[[Tensor, Tensor, Tensor], Tensor], labels: Tensor, w: float):
    """``DiffusionCondition.py:83-85``: eps = (1+w) eps(labels) - w eps(0)."""
    def f(x, t):
        e = model_fn3(x, t, labels)
        n = model_fn3(x, t, torch.zeros_like(labels))
        return (1.0 + w) * e - w * n
    return f


# --------------------------------------------------------------------------- verifiers
def oracle_score(images: Tensor) -> float:
    """``verifier.py:60-63`` (dataset_stats=None)."""
    variance = torch.var(images.flatten(1), dim=1).mean().item()
    return 1.0 / (1.0 + variance)


def selfsup_score(images: Tensor) -> float:
    """``verifier.py:219-248`` without reference features (B=1 gives NaN)."""
    f = F.adaptive_avg_pool2d(images, (8, 8)).flatten(1)
    f = F.normalize(f, dim=-1)
    sim = f @ f.T
    mask = ~torch.eye(len(f), dtype=torch.bool)
    return sim[mask].mean().item()


def aesthetic_score(images: Tensor) -> float:
    """``verifier.py:277-287``: data-dependent rescale then 2 * mean per-image std."""
    if images.min() < 0:
        images = (images + 1) / 2
    cd = torch.std(images.flatten(1), dim=1).mean()
    ct = torch.std(images.view(len(images), -1), dim=1).mean()
    return (cd + ct).item()


def oracle_stats_score(images: Tensor) -> float:
    """``verifier.py:65-66``: with dataset_stats the reference returns the plain mean."""
    return torch.mean(images).item()


def selfsup_paired_score(images: Tensor, reference_features: Tensor) -> float:
    """``verifier.py:232-240`` with reference features: per-image cosine, then .item()."""
    f = F.normalize(F.adaptive_avg_pool2d(images, (8, 8)).flatten(1), dim=-1)
    r = F.normalize(reference_features, dim=-1)
    return torch.sum(f * r, dim=-1).item()


VERIFIERS = {"oracle": oracle_score, "selfsup": selfsup_score, "aesthetic": aesthetic_score}


# --------------------------------------------------------------------------- search
def random_search(n: int, noise_shape: Tuple[int, ...], denoise_fn, verifier_fn):
    """``search_algorithm.py:54-83``; also returns all scores (collected at :76)."""
    best_noise, best_score, scores = None, float("-inf"), []
    for i in range(n):
        noise = torch.randn(noise_shape)
        with torch.no_grad():
            den = denoise_fn(noise)
        s = verifier_fn(den)
        scores.append(s)
        if s > best_score:
            best_score, best_noise = s, noise.clone()
    return best_noise, best_score, scores


def zero_order_search(initial: Tensor, n_neighbors: int, lambda_radius: float, n_iterations: int,
                      denoise_fn, verifier_fn):
    """``search_algorithm.py:142-231``."""
    cur = initial.clone()
    best_noise, best_score = initial.clone(), float("-inf")
    hist = {"scores": [], "candidates_per_iter": []}
    for _ in range(n_iterations):
        neigh = [cur + torch.randn_like(cur) * (1 - lambda_radius) for _ in range(n_neighbors)]
        its, bc, bcs = [], None, float("-inf")
        for nb in neigh:
            with torch.no_grad():
                den = denoise_fn(nb)
            s = verifier_fn(den)
            its.append(s)
            if s > bcs:
                bcs, bc = s, nb.clone()
        hist["scores"].append(its)
        hist["candidates_per_iter"].append(len(neigh))
        if bcs > best_score:
            best_score, best_noise, cur = bcs, bc.clone(), bc.clone()
    return best_noise, best_score, hist


def path_search(initial: Tensor, n_paths: int, injection_step: int, noise_scale: float, denoise_fn, verifier_fn):
    """``search_algorithm.py:292-336`` (the injection is a placeholder there)."""
    best_noise, best_score = initial.clone(), float("-inf")
    hist = {"scores": [], "injection_points": []}
    for _ in range(n_paths):
        pert = initial + torch.randn_like(initial) * noise_scale
        with torch.no_grad():
            den = denoise_fn(pert)
        s = verifier_fn(den)
        hist["scores"].append(s)
        hist["injection_points"].append(injection_step)
        if s > best_score:
            best_score, best_noise = s, pert.clone()
    return best_noise, best_score, hist


# --------------------------------------------------------------------------- counter-based noise
def philox_normal(seed: int, step: int, idx) -> Tensor:
    """The throughput mode's noise z(seed, step, element) -- NOT a reference function: the
    reference draws ``torch.randn_like`` from the global generator (``Diffusion.py:96``), and
    parity with it goes through injected noise. This restates itsd's own generator
    (``csrc/kernels.hip`` philox_normal: Philox4x32-10, Salmon et al. SC'11, counter
    (idx_lo, idx_hi, step, 0x1d5a1), key (seed_lo, seed_hi); Box-Muller on words 0, 1) in
    numpy so that Philox-mode GPU runs can be checked step by step against this oracle."""
    import numpy as np

    M32 = np.uint64(0xFFFFFFFF)
    idx = np.asarray(idx, dtype=np.uint64)
    c0 = idx & M32
    c1 = idx >> np.uint64(32)
    c2 = np.full_like(c0, np.uint64(step & 0xFFFFFFFF))
    c3 = np.full_like(c0, np.uint64(0x1D5A1))
    k0 = np.uint64(seed & 0xFFFFFFFF)
    k1 = np.uint64((seed >> 32) & 0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c0
        p1 = np.uint64(0xCD9E8D57) * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & M32
        hi1, lo1 = p1 >> np.uint64(32), p1 & M32
        n0 = hi1 ^ c1 ^ k0
        n2 = hi0 ^ c3 ^ k1
        c0, c1, c2, c3 = n0, lo1, n2, lo0
        k0 = (k0 + np.uint64(0x9E3779B9)) & M32
        k1 = (k1 + np.uint64(0xBB67AE85)) & M32
    u1 = ((c0 >> np.uint64(8)).astype(np.float32) + np.float32(0.5)) * np.float32(1.0 / 16777216.0)
    u2 = (c1 >> np.uint64(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    z = np.sqrt(np.float32(-2.0) * np.log(u1)) * np.cos(np.float32(6.283185307179586) * u2)
    return torch.from_numpy(z.astype(np.float32))
