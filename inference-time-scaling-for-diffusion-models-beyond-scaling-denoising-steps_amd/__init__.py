"""itsd — MI355X-native search-over-noise diffusion sampler.

Drop-in for the reference's hot path: the DDPM/CFG
ancestral sampler (``Diffusion/Diffusion.py``, ``DiffusionFreeGuidence/DiffusionCondition.py``)
driving N candidate noises through T UNet steps (``Diffusion/Model.py``), scored by
``search/verifier.py`` and selected by ``search/search_algorithm.py``.

Compute runs in ``libitsd_hip.so`` (hand-written gfx950 HIP kernels behind a C ABI,
``include/itsd.h``); this package is the host-side mirror of the reference's Python
interface. Import via the ``itsd`` shim at the repository root.
"""
from .arch import ARCH_A, ARCH_C, ARCH_TINY, ARCH_TINY_CFG, UNetArch  # noqa: F401

__all__ = ["UNetArch", "ARCH_A", "ARCH_C", "ARCH_TINY", "ARCH_TINY_CFG"]
