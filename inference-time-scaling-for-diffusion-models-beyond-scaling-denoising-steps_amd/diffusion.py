"""Ancestral samplers with the reference interface.

* ``GaussianDiffusionSampler``     <- ``Diffusion/Diffusion.py:50-102``
* ``CondGaussianDiffusionSampler`` <- ``DiffusionFreeGuidence/DiffusionCondition.py:56-105``
  (also exported as ``itsd.diffusion_condition.GaussianDiffusionSampler``)

``forward`` runs the whole T-step loop inside libitsd_hip (``itsd_sampler_run``):
one hipGraph per denoising step replayed T times, the step counter in device
memory, noise from counter-based Philox (or injected, for parity), and the NaN
check of ``Diffusion.py:100`` reduced to one device flag read at the end.

RNG: the reference draws ``torch.randn_like`` from the global generator each step.
Here the per-run Philox seed is drawn from the global torch generator, so runs
are deterministic under ``torch.manual_seed``; bit-identical noise to the reference
is available by passing ``noise=`` (see ``reference_noise_plan``).
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch

from .schedule import make_schedule


def _extract(v: torch.Tensor, t: torch.Tensor, ndim: int) -> torch.Tensor:
    """``Diffusion.py:9-16``."""
    out = torch.gather(v.to(t.device), index=t.long(), dim=0).float()
    return out.view([t.shape[0]] + [1] * (ndim - 1))


def _draw_seed() -> int:
    return int(torch.randint(0, 2 ** 62, (1,)).item())


class GaussianDiffusionSampler:
    def __init__(self, model, beta_1: float, beta_T: float, T: int, w: float = 0.0):
        self.model = model
        self.T = int(T)
        self.w = float(w)
        self.sched = make_schedule(beta_1, beta_T, T)
        # the reference's registered buffers (Diffusion.py:57-65)
        self.betas = self.sched.betas
        self.coeff1 = self.sched.coeff1
        self.coeff2 = self.sched.coeff2
        self.posterior_var = self.sched.posterior_var
        self._sched_args = (self.sched.coeff1_f32, self.sched.coeff2_f32, self.sched.sqrt_var_f32, self.w)
        self.last_seed = None  # Philox key of the last run (set by run)

    def to(self, *args, **kwargs):
        if args or "device" in kwargs:
            self.model.to(*args, **kwargs)
        return self

    def eval(self):
        return self

    def _native(self, n: int):
        nat = self.model.native(n)
        if getattr(nat, "_sched_args", None) is not self._sched_args:
            nat.set_schedule(*self._sched_args)
            nat._sched_args = self._sched_args
        return nat

    # --- reference API
    def predict_xt_prev_mean_from_eps(self, x_t, t, eps):
        assert x_t.shape == eps.shape
        return _extract(self.coeff1, t, x_t.ndim) * x_t - _extract(self.coeff2, t, x_t.ndim) * eps

    def p_mean_variance(self, x_t: torch.Tensor, t: torch.Tensor, labels: Optional[torch.Tensor] = None):
        """``Diffusion.py:74-82`` (one UNet call through the native forward)."""
        var = _extract(self.sched.var, t, x_t.ndim)
        if labels is None:
            eps = self.model(x_t, t)
        else:
            e = self.model(x_t, t, labels)
            ne = self.model(x_t, t, torch.zeros_like(labels))
            eps = (1.0 + self.w) * e - self.w * ne
        return self.predict_xt_prev_mean_from_eps(x_t, t, eps), var

    def run(self, x: torch.Tensor, t_begin: Optional[int] = None, t_end: int = 0, labels=None, seed=None,
            noise: Optional[torch.Tensor] = None, noise_offset: int = 0, graph: bool = True, clip=None,
            sync: bool = True) -> torch.Tensor:
        """In-place steps t_begin..t_end on a contiguous fp32 device tensor x."""
        t_begin = self.T - 1 if t_begin is None else int(t_begin)
        if clip is None:
            clip = t_end == 0
        if seed is None and noise is None:
            seed = _draw_seed()
        self.last_seed = seed  # the Philox key of this run (None with injected noise)
        if noise is not None:
            noise = noise.to(x.device, torch.float32).contiguous()
            if noise.shape[0] < t_begin + 1 or noise[0].numel() != x.numel():
                raise ValueError("noise must be [T, *x.shape] indexed by step t")
        if labels is not None:
            labels = labels.flatten().to(x.device, torch.int32).contiguous()
        nat = self._native(x.shape[0])
        nat.run(x, t_begin, t_end, seed or 0, noise=noise, labels=labels, noise_offset=noise_offset, graph=graph,
                clip=clip, sync=sync)
        return x

    def forward(self, x_T: torch.Tensor, noise: Optional[torch.Tensor] = None, seed: Optional[int] = None,
                graph: bool = True) -> torch.Tensor:
        """Algorithm 2 (``Diffusion.py:84-102``): returns clip(x_0, -1, 1)."""
        x = x_T.to(self.model.device, torch.float32).clone().contiguous()
        return self.run(x, labels=None, seed=seed, noise=noise, graph=graph)

    __call__ = forward

    def reference_noise(self, shape: Sequence[int]) -> torch.Tensor:
        """The T-1 draws one reference sampler call takes from the global CPU generator
        (``Diffusion.py:94-96``: ``randn_like`` at t = T-1 .. 1), as [T, *shape] by step t."""
        z = [torch.randn(tuple(shape)) for _ in range(self.T - 1)]
        return torch.stack(z + [torch.zeros(tuple(shape))]).flip(0)

    def denoise_fn(self, reference_rng: bool = True, labels: Optional[torch.Tensor] = None):
        """A ``denoise_fn(noise, show_progress, **kw)`` for the sequential search API
        (``search_algorithm.py:71``). reference_rng: each call consumes the reference's
        per-step draws from the global generator (bit-identical candidates to the reference
        loop under ``torch.manual_seed``); otherwise Philox seeded from that generator."""

        def fn(noise: torch.Tensor, show_progress: bool = False, **kw) -> torch.Tensor:
            z = self.reference_noise(noise.shape) if reference_rng else None
            x = noise.to(self.model.device, torch.float32).clone().contiguous()
            return self.run(x, labels=labels, noise=z)

        return fn


class CondGaussianDiffusionSampler(GaussianDiffusionSampler):
    """``DiffusionCondition.py:56``: guided eps = (1+w) eps(x,t,y) - w eps(x,t,0)."""

    def __init__(self, model, beta_1: float, beta_T: float, T: int, w: float = 0.0):
        super().__init__(model, beta_1, beta_T, T, w)

    def forward(self, x_T: torch.Tensor, labels: torch.Tensor, noise: Optional[torch.Tensor] = None,
                seed: Optional[int] = None, graph: bool = True) -> torch.Tensor:
        x = x_T.to(self.model.device, torch.float32).clone().contiguous()
        return self.run(x, labels=labels, seed=seed, noise=noise, graph=graph)

    __call__ = forward

    def denoise_fn(self, reference_rng: bool = True, labels: Optional[torch.Tensor] = None):
        if labels is None:
            raise ValueError("the guided sampler's denoise_fn needs labels")
        return super().denoise_fn(reference_rng, labels)


def reference_noise_plan(shape: Sequence[int], T: int, n_runs: int = 1) -> Tuple[torch.Tensor, torch.Tensor]:
    """The exact draws the reference consumes from the global CPU generator for
    ``n_runs`` back-to-back ``randn(shape)`` + T-step sampler runs (RandomSearch order,
    ``search_algorithm.py:67`` then ``Diffusion.py:96`` for t = T-1..1).

    Returns (x_T [n_runs, *shape], noise [T, n_runs*shape[0], ...]) batched so that one
    ``sampler.run`` over all runs reproduces the reference's candidates bit-for-bit
    (noise[t] is the draw used at step t; noise[0] is unused)."""
    shape = tuple(shape)
    xs, zs = [], []
    for _ in range(n_runs):
        xs.append(torch.randn(shape))
        zs.append(torch.stack([torch.randn(shape) for _ in range(T - 1)] + [torch.zeros(shape)]).flip(0))
    x_T = torch.stack(xs)
    noise = torch.stack(zs, dim=1).reshape(T, n_runs * shape[0], *shape[1:])
    return x_T, noise
