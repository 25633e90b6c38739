"""Verifiers with the reference interface (``search/verifier.py``), scored on the GPU.

``score(images) -> float`` keeps the reference's one-candidate semantics;
``score_batch(images, n_cand) -> Tensor[n_cand]`` scores every candidate of a
batched round in one ``itsd_verify`` launch (one block per candidate), which is
what the batched search engine uses. CLIP-based verifiers (``verifier.py:69-188,
290-388``) need downloaded weights and are out of scope.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import runtime as rt


def _dev(images: torch.Tensor) -> torch.Tensor:
    if not images.is_cuda:
        images = images.cuda()
    return images.to(torch.float32).contiguous()


class _NativeVerifier:
    kind: int

    def score_batch(self, images: torch.Tensor, n_cand: int) -> torch.Tensor:
        return rt.verify(self.kind, _dev(images), n_cand)

    def __call__(self, images, **kwargs) -> float:
        return self.score(images)


class OracleVerifier(_NativeVerifier):
    """``verifier.py:30-66``: 1/(1 + mean_b var(x_b)) when no dataset stats are given."""

    kind = rt.VERIFY_ORACLE

    def __init__(self, dataset_stats: Optional[Dict[str, np.ndarray]] = None):
        self.dataset_stats = dataset_stats

    def score_batch(self, images: torch.Tensor, n_cand: int) -> torch.Tensor:
        # with dataset stats the reference's TODO branch scores the plain mean (verifier.py:66)
        kind = rt.VERIFY_ORACLE if self.dataset_stats is None else rt.VERIFY_MEAN
        return rt.verify(kind, _dev(images), n_cand)

    def score(self, images: torch.Tensor, labels: Optional[torch.Tensor] = None) -> float:
        return float(self.score_batch(images, 1)[0].item())


class SelfSupervisedVerifier(_NativeVerifier):
    """``verifier.py:191-248``: mean off-diagonal cosine of 8x8-pooled features
    (NaN for a single image, as the reference)."""

    kind = rt.VERIFY_SELFSUP

    def __init__(self, denoising_features: Optional[torch.Tensor] = None):
        self.denoising_features = denoising_features

    def extract_features(self, images: torch.Tensor) -> torch.Tensor:
        return F.adaptive_avg_pool2d(images, (8, 8)).flatten(1)

    def score(self, images: torch.Tensor, reference_features: Optional[torch.Tensor] = None) -> float:
        if reference_features is not None:  # verifier.py:237-240: per-image cosine, then .item()
            images = _dev(images)
            if images.shape[0] != 1:  # the reference's .item() of a b-vector raises the same way
                raise RuntimeError(f"a Tensor with {images.shape[0]} elements cannot be converted to Scalar")
            return float(rt.verify_paired(images, reference_features.reshape(1, -1))[0].item())
        return float(self.score_batch(images, 1)[0].item())


class AestheticPredictor(_NativeVerifier):
    """``verifier.py:251-287``: (x+1)/2 if the candidate has negatives, then 2 * mean std."""

    kind = rt.VERIFY_AESTHETIC

    def __init__(self, device: str = "cuda"):
        self.device = device
        self.model = None

    def score(self, images: torch.Tensor) -> float:
        return float(self.score_batch(images, 1)[0].item())


VERIFIERS = {"oracle": OracleVerifier, "selfsup": SelfSupervisedVerifier, "aesthetic": AestheticPredictor}
