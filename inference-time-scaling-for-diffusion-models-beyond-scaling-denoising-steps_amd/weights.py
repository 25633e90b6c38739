"""Weights: synthetic recipes and reference-checkpoint loading.

The reference cannot run without a checkpoint (``Diffusion/Train.py:816-818``);
there is no network here to fetch one, so benchmarks and parity tests use a
seeded synthetic recipe. The reference's own init (``xavier_uniform_`` with
gain 1e-5 on each ResBlock's last conv and on the tail conv, ``Model.py:200,262``)
makes the UNet output eps with std ~7.6e-6 (SURVEY.md finding 5), which would make
parity nearly vacuous, so the default recipe ("gauss") is non-degenerate:

* conv / linear weights ~ N(0, 1/fan_in); biases ~ 0.05 N(0, 1)
* GroupNorm weight ~ 1 + 0.1 N(0, 1), bias ~ 0.1 N(0, 1)
* ``time_embedding.freq_coeffs`` = the reference buffer formula (``Model.py:33-34``)
* CFG tables: the sinusoid table of ``ModelCondition.py:28-35``; label table
  N(0, 1) with row 0 zeroed (``padding_idx=0``, ``ModelCondition.py:54``).

Draws happen on a CPU ``torch.Generator`` in key order, so a (arch, seed) pair
names one exact tensor set on every machine.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict

import torch

from .arch import UNetArch, param_specs


def freq_coeffs(d_model: int) -> torch.Tensor:
    """``Model.py:33-34``: exp(-(arange(0,d,2)/d * ln 10000))."""
    emb = torch.arange(0, d_model, step=2).float() / d_model * math.log(10000)
    return torch.exp(-emb)


def sinusoid_table(T: int, d_model: int) -> torch.Tensor:
    """``ModelCondition.py:28-35`` (note: no ``.float()`` before the division there,
    arange is int64 so true division gives float32 as well)."""
    emb = torch.arange(0, d_model, step=2) / d_model * math.log(10000)
    emb = torch.exp(-emb)
    pos = torch.arange(T).float()
    emb = pos[:, None] * emb[None, :]
    emb = torch.stack([torch.sin(emb), torch.cos(emb)], dim=-1)
    return emb.view(T, d_model)


def synthetic_state_dict(a: UNetArch, seed: int = 0, recipe: str = "gauss") -> "OrderedDict[str, torch.Tensor]":
    specs = param_specs(a)
    g = torch.Generator().manual_seed(int(seed))
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    for name, shape in specs.items():
        if name == "time_embedding.freq_coeffs":
            sd[name] = freq_coeffs(a.ch)
            continue
        if a.cfg and name == "time_embedding.timembedding.0.weight":
            sd[name] = sinusoid_table(a.T, a.ch)
            continue
        if a.cfg and name == "cond_embedding.condEmbedding.0.weight":
            t = torch.randn(shape, generator=g)
            t[0].zero_()
            sd[name] = t
            continue
        is_gn = (".block1.0." in name or ".block2.0." in name or ".group_norm." in name
                 or name.startswith("tail.0."))
        if name.endswith(".weight"):
            if is_gn:
                sd[name] = 1.0 + 0.1 * torch.randn(shape, generator=g)
            else:
                if recipe == "gauss":
                    fan_in = int(torch.tensor(shape[1:]).prod()) if len(shape) > 1 else shape[0]
                    if name.endswith(".t.weight"):  # ConvTranspose2d [Cin, Cout, k, k]: fan-in over Cin*k*k/4 taps
                        fan_in = shape[0] * shape[2] * shape[3] // 4
                    sd[name] = torch.randn(shape, generator=g) / math.sqrt(fan_in)
                elif recipe == "xavier":
                    w = torch.empty(shape)
                    fan_in = int(torch.tensor(shape[1:]).prod())
                    fan_out = shape[0] * (int(torch.tensor(shape[2:]).prod()) if len(shape) > 2 else 1)
                    bound = math.sqrt(6.0 / (fan_in + fan_out))
                    gain = 1e-5 if (name.endswith("block2.3.weight") or name == "tail.2.weight"
                                    or name.endswith("attn.proj.weight")) else 1.0
                    w.uniform_(-bound * gain, bound * gain, generator=g)
                    sd[name] = w
                else:
                    raise ValueError(f"unknown weight recipe {recipe!r}")
        else:  # bias
            if is_gn:
                sd[name] = 0.1 * torch.randn(shape, generator=g)
            else:
                sd[name] = (0.05 * torch.randn(shape, generator=g)) if recipe == "gauss" else torch.zeros(shape)
    return sd


def load_reference_checkpoint(path: str) -> "OrderedDict[str, torch.Tensor]":
    """Load a reference ``torch.save(model.state_dict())`` file (``Train.py:717``).

    Only the safe loader is used (``weights_only=True``); a ``module.`` prefix
    left by DataParallel is stripped as the reference does (``Train.py:564-571``).
    """
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
        sd = sd["state_dict"]
    out: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    for k, v in sd.items():
        out[k[len("module."):] if k.startswith("module.") else k] = v
    return out


def check_state_dict(a: UNetArch, sd: Dict[str, torch.Tensor]) -> None:
    """Raise ``KeyError``/``ValueError`` the way ``load_state_dict(strict=True)`` would."""
    specs = param_specs(a)
    missing = [k for k in specs if k not in sd]
    unexpected = [k for k in sd if k not in specs]
    if missing or unexpected:
        raise KeyError(f"state_dict mismatch: missing={missing[:8]} unexpected={unexpected[:8]}")
    for k, shp in specs.items():
        if tuple(sd[k].shape) != tuple(shp):
            raise ValueError(f"size mismatch for {k}: checkpoint {tuple(sd[k].shape)} vs model {tuple(shp)}")
