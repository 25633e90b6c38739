"""UNet facades with the reference constructor signatures and state_dict surface.

* ``UNet``     <- ``Diffusion/Model.py:212`` ``UNet(T, ch, ch_mult, attn, num_res_blocks, dropout)``
* ``CondUNet`` <- ``DiffusionFreeGuidence/ModelCondition.py:164``
  ``UNet(T, num_labels, ch, ch_mult, num_res_blocks, dropout)`` (also exported as
  ``itsd.model_condition.UNet``)

Forward runs entirely in libitsd_hip (``itsd_unet_forward``). The facade keeps the
fp32 state_dict on the host (for re-packing when the batch capacity grows) and
creates the native handle lazily; there is no PyTorch compute fallback.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Optional

import torch

from . import runtime as rt
from .arch import ARCH_CFG, ARCH_DDPM, UNetArch
from .weights import check_state_dict, synthetic_state_dict

_PREC = {"fp32": rt.PREC_FP32, "bf16": rt.PREC_BF16}


def _round_up_pow2(n: int) -> int:
    p = 1
    while p < n:
        p <<= 1
    return p


class _NativeModule:
    arch: UNetArch

    def _init_common(self, arch: UNetArch, precision: str, weights: str, seed: int, device):
        if precision not in _PREC:
            raise ValueError(f"precision must be one of {sorted(_PREC)}")
        self.arch = arch
        self.precision = precision
        self.device = torch.device(device) if device is not None else torch.device("cuda", 0)
        # Reference modules initialise their own weights (xavier, Model.py:194-201,258-262);
        # "xavier" mirrors that, "gauss" is the non-degenerate benchmarking recipe.
        self._sd: "OrderedDict[str, torch.Tensor]" = synthetic_state_dict(arch, seed, recipe=weights)
        self._native: Optional[rt.NativeUNet] = None
        self.training = False

    # --- nn.Module-like surface used by the reference call sites
    def state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        return OrderedDict((k, v.clone()) for k, v in self._sd.items())

    def load_state_dict(self, state_dict: Dict[str, torch.Tensor], strict: bool = True):
        sd = OrderedDict((k[7:] if k.startswith("module.") else k, v) for k, v in state_dict.items())
        if strict:
            check_state_dict(self.arch, sd)
        merged = OrderedDict(self._sd)
        for k, v in sd.items():
            if k in merged:
                merged[k] = v.detach().to("cpu", torch.float32).clone()
        self._sd = merged
        self._release()
        return self

    def eval(self):
        self.training = False
        return self

    def train(self, mode: bool = True):
        if mode:
            raise NotImplementedError("itsd is an inference-only sampler (training is out of scope)")
        return self

    def to(self, device=None, *args, **kwargs):
        if device is not None:
            dev = torch.device(device)
            if dev.type != "cuda":
                raise ValueError("itsd runs on the GPU only (HIP); no CPU execution path")
            if dev.index is None:
                dev = torch.device("cuda", torch.cuda.current_device())
            if dev != self.device:
                self._release()
            self.device = dev
        return self

    def parameters(self):
        return iter(self._sd.values())

    def _release(self):
        if self._native is not None:
            self._native.close()
            self._native = None

    def native(self, n: int) -> rt.NativeUNet:
        """The native handle, (re)created with capacity >= n."""
        if self._native is None or self._native.max_batch < n:
            cap = max(n, 8 if self._native is None else 2 * self._native.max_batch)
            cap = _round_up_pow2(cap)
            sched = getattr(self._native, "_sched_args", None)
            self._release()
            torch.cuda.set_device(self.device)
            self._native = rt.NativeUNet(self.arch, self._sd, cap, _PREC[self.precision], self.device.index or 0)
            if sched is not None:
                self._native.set_schedule(*sched)
                self._native._sched_args = sched
        return self._native

    def reserve(self, n: int) -> "rt.NativeUNet":
        """Pre-size the workspace for batch n (avoids a re-pack inside a timed loop)."""
        return self.native(n)

    def _prep(self, x: torch.Tensor, t) -> tuple:
        if x.dim() != 4 or x.shape[1] != 3 or x.shape[2] != self.arch.img_size or x.shape[3] != self.arch.img_size:
            raise ValueError(f"expected x of shape [B,3,{self.arch.img_size},{self.arch.img_size}], got {tuple(x.shape)}")
        x = x.to(self.device, torch.float32).contiguous()
        if not torch.is_tensor(t):
            t = torch.full((x.shape[0],), int(t), dtype=torch.int32)
        t = t.flatten().to(self.device, torch.int32).contiguous()
        if t.numel() != x.shape[0]:
            raise ValueError("t must have one entry per image")
        return x, t


class UNet(_NativeModule):
    """``Diffusion/Model.py:212``. Extra keyword arguments: img_size, precision
    ("fp32" parity mode / "bf16" throughput mode), weights recipe, seed, device."""

    def __init__(self, T, ch, ch_mult, attn, num_res_blocks, dropout, img_size: int = 32, precision: str = "fp32",
                 weights: str = "xavier", seed: int = 0, device=None):
        arch = UNetArch(ch=ch, ch_mult=tuple(ch_mult), attn=tuple(attn), num_res_blocks=num_res_blocks, T=T,
                        img_size=img_size, kind=ARCH_DDPM)
        self.dropout = dropout  # identity at inference (nn.Dropout in eval, Model.py:182)
        self._init_common(arch, precision, weights, seed, device)

    def forward(self, x: torch.Tensor, t) -> torch.Tensor:
        x, t = self._prep(x, t)
        eps = torch.empty_like(x)
        self.native(x.shape[0]).forward(x, t, None, eps)
        return eps

    __call__ = forward


class CondUNet(_NativeModule):
    """``DiffusionFreeGuidence/ModelCondition.py:164``."""

    def __init__(self, T, num_labels, ch, ch_mult, num_res_blocks, dropout, img_size: int = 32,
                 precision: str = "fp32", weights: str = "gauss", seed: int = 0, device=None):
        arch = UNetArch(ch=ch, ch_mult=tuple(ch_mult), attn=(), num_res_blocks=num_res_blocks, T=T,
                        img_size=img_size, kind=ARCH_CFG, num_labels=num_labels)
        self.dropout = dropout
        self._init_common(arch, precision, weights, seed, device)

    def forward(self, x: torch.Tensor, t, labels, return_representation: bool = False):
        """``ModelCondition.py:206-235``: eps, or (eps, h) with h the pre-tail activation
        (``last_representation``, NCHW fp32 [B, ch * ch_mult[0], H, W]) when return_representation."""
        x, t = self._prep(x, t)
        lab = labels.flatten().to(self.device, torch.int32).contiguous()
        if int(lab.min()) < 0 or int(lab.max()) > self.arch.num_labels:
            raise IndexError("label out of range for the condition embedding table")
        if int(t.max()) >= self.arch.T or int(t.min()) < 0:
            raise IndexError("t out of range for the time-embedding table (ModelCondition.py:38)")
        eps = torch.empty_like(x)
        nat = self.native(x.shape[0])
        nat.forward(x, t, lab, eps)
        if return_representation:
            a = self.arch
            return eps, nat.representation(x.shape[0], a.ch * a.ch_mult[0], a.img_size, x.device)
        return eps

    __call__ = forward
