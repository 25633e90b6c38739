"""DDPM schedule tables (host, fp64 -> fp32), exactly as the reference builds them.

``Diffusion/Diffusion.py:57-65`` (twin ``DiffusionCondition.py:68-73``):
betas = linspace(beta_1, beta_T, T) computed in fp32 then ``.double()``;
coeff1 = sqrt(1/alpha); coeff2 = coeff1 (1-alpha)/sqrt(1-alpha_bar);
posterior_var = beta (1-alpha_bar_prev)/(1-alpha_bar).
``p_mean_variance`` (``Diffusion.py:74-77``) uses var = cat([posterior_var[1:2], betas[1:]]).
``extract`` (``:9-16``) gathers and casts to fp32, so the device consumes the
fp32 casts; ``torch.sqrt(var)`` (``:99``) is an fp32 sqrt of the fp32 var, which
is precomputed here bit-for-bit with torch.
"""
from __future__ import annotations

import dataclasses

import torch
import torch.nn.functional as F


@dataclasses.dataclass
class Schedule:
    T: int
    beta_1: float
    beta_T: float
    betas: torch.Tensor          # fp64 [T]
    coeff1: torch.Tensor         # fp64 [T]
    coeff2: torch.Tensor         # fp64 [T]
    posterior_var: torch.Tensor  # fp64 [T]
    var: torch.Tensor            # fp64 [T]  (cat([posterior_var[1:2], betas[1:]]))

    @property
    def coeff1_f32(self) -> torch.Tensor:
        return self.coeff1.float()

    @property
    def coeff2_f32(self) -> torch.Tensor:
        return self.coeff2.float()

    @property
    def sqrt_var_f32(self) -> torch.Tensor:
        return torch.sqrt(self.var.float())


def make_schedule(beta_1: float, beta_T: float, T: int) -> Schedule:
    betas = torch.linspace(beta_1, beta_T, T).double()
    alphas = 1.0 - betas
    alphas_bar = torch.cumprod(alphas, dim=0)
    alphas_bar_prev = F.pad(alphas_bar, [1, 0], value=1)[:T]
    coeff1 = torch.sqrt(1.0 / alphas)
    coeff2 = coeff1 * (1.0 - alphas) / torch.sqrt(1.0 - alphas_bar)
    posterior_var = betas * (1.0 - alphas_bar_prev) / (1.0 - alphas_bar)
    var = torch.cat([posterior_var[1:2], betas[1:]])
    return Schedule(T, float(beta_1), float(beta_T), betas, coeff1, coeff2, posterior_var, var)
