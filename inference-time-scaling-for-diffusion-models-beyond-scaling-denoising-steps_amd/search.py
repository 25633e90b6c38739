"""Search over initial noise (``search/search_algorithm.py``).

Two layers:

1. ``RandomSearch`` / ``ZeroOrderSearch`` / ``PathSearch`` keep the reference
   constructors, ``search`` signatures, return values, ``nfes`` bookkeeping and the
   sequential candidate loop, calling the user's ``denoise_fn`` / ``verifier_fn``
   (``search_algorithm.py:18-340``). With ``batched=True`` (and a ``sampler=`` plus an
   itsd verifier) a round's candidates are instead denoised as ONE batch.

2. ``SearchEngine`` is the MI355X-native round executor: the round's N candidates
   are sharded over the ranks of a ``torch.distributed`` group (one process per
   GPU), each rank generates its candidates' noise from (seed, round, GLOBAL index)
   by Philox, runs the whole T-step sampler in libitsd_hip, scores its candidates
   on the GPU, and ONE all_gather of the N fp64 scores per round gives every rank
   the same argmax (strict '>' scan order = lowest global index on ties, NaN never
   wins, ``search_algorithm.py:79``). The winner's noise is regenerated locally from
   its global index, so no noise ever crosses xGMI; the winner's denoised image is
   kept by its owner rank and broadcast once when the search ends.

   ``noise="reference"`` is the parity mode (one process): every round draws its
   candidates and the sampler's per-step noise from torch's global CPU generator in
   exactly the order the reference's sequential loops consume them, and feeds them
   to the batched sampler as injected noise -- the batched search then reproduces
   the reference's scores, argmax and best noise bit for bit under
   ``torch.manual_seed`` -- of a reference run with ``device="cpu"`` (its default
   ``device="cuda"`` would draw from the CUDA generator); small rounds only.
"""
from __future__ import annotations

import dataclasses
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import runtime as rt

_STREAM_XT = 0xF0000000      # Philox stream ids (the sampler uses stream id = t < T)
_STREAM_PERTURB = 0xE0000000
_STREAM_INIT = 0xD0000000    # the initial pivot of zero-order / path search


def strict_argmax(scores: torch.Tensor) -> Tuple[int, float]:
    """The reference's ``if score > best_score`` scan from -inf (``search_algorithm.py:79,
    193, 329``): the first maximum wins ties and a NaN score never wins. Returns
    (-1, -inf) when no score beats -inf (the reference then keeps its initial best)."""
    sc = torch.nan_to_num(scores.detach().double().cpu(), nan=float("-inf"))
    if sc.numel() == 0 or not bool((sc > float("-inf")).any()):
        return -1, float("-inf")
    i = int(torch.argmax(sc).item())  # first occurrence of the maximum
    return i, float(sc[i])


# --------------------------------------------------------------------------- engine
@dataclasses.dataclass
class RoundResult:
    scores: torch.Tensor          # [N] fp64 (all candidates, every rank)
    best_index: int               # global index of the round's best candidate (-1: none)
    best_score: float
    local_images: torch.Tensor    # this rank's denoised candidates [n_local*B,3,H,W]
    g0: int = 0                   # global index of this rank's first candidate


class ReferenceNoise:
    """The reference's random draws, in its order, from torch's global CPU generator.

    * random (``search_algorithm.py:65-75``): per candidate ``randn(shape)``, then the
      sampler's T-1 ``randn_like`` (``Diffusion.py:94-96``, t = T-1 .. 1);
    * zero_order (``:156-187``, ``_sample_neighbors`` ``:221-229``): all neighbours
      ``pivot + randn_like(pivot) * (1 - lambda)`` first, then per neighbour T-1 draws;
    * path (``:305-318``): per path ``initial + randn_like(initial) * scale``, then T-1.

    Returns (x_T [n*B,...], noise [T, n*B, ...]) on the CPU; noise[t] feeds step t.

    Parity is defined against a reference run with ``device="cpu"`` (what search_T5.npz
    holds): the reference's default ``device="cuda"`` draws from the CUDA generator instead.
    The whole [T, n*B, ...] plan is materialised on the host and copied to the device, so it
    is meant for parity-sized rounds: above ``MAX_ELEMENTS`` it refuses (use Philox mode)."""

    MAX_ELEMENTS = 1 << 28  # 1 GiB of fp32 noise per round

    def __init__(self, T: int):
        self.T = int(T)

    def _steps(self, shape) -> torch.Tensor:
        z = [torch.randn(shape) for _ in range(self.T - 1)]
        return torch.stack(z + [torch.zeros(shape)]).flip(0)  # [T][shape], index = step t

    def round(self, kind: str, n: int, shape, pivot: Optional[torch.Tensor] = None, scale: float = 1.0):
        shape = tuple(shape)
        total = self.T * n * int(torch.Size(shape).numel())
        if total > self.MAX_ELEMENTS:
            raise ValueError(f"reference-order noise plan of {total} elements (T={self.T}, n={n}) exceeds "
                             f"{self.MAX_ELEMENTS}: parity mode is for small rounds, use noise='philox'")
        xs, zs = [], []
        if kind == "zero_order":
            p = pivot.detach().cpu().float()
            xs = [p + torch.randn_like(p) * scale for _ in range(n)]
            zs = [self._steps(shape) for _ in range(n)]
        else:
            for _ in range(n):
                if kind == "random":
                    xs.append(torch.randn(shape))
                else:
                    p = pivot.detach().cpu().float()
                    xs.append(p + torch.randn_like(p) * scale)
                zs.append(self._steps(shape))
        x_T = torch.cat(xs)
        noise = torch.stack(zs, dim=1).reshape(self.T, n * shape[0], *shape[1:])
        return x_T, noise


class SearchEngine:
    """Batched, sharded search rounds over a sampler + native verifier."""

    def __init__(self, sampler, verifier, seed: int = 0, group=None, graph: bool = True, noise: str = "philox"):
        if not hasattr(verifier, "kind"):
            raise TypeError("SearchEngine needs an itsd verifier (OracleVerifier / SelfSupervisedVerifier / "
                            "AestheticPredictor); wrap custom scorers in the sequential API")
        if noise not in ("philox", "reference"):
            raise ValueError("noise must be 'philox' (sharded, counter-based) or 'reference' (parity mode)")
        self.sampler = sampler
        self.verifier = verifier
        self.seed = int(seed)
        self.group = group
        self.graph = graph
        # with a process group (even of one rank) the round protocol runs its collectives: the
        # code path of an N-GPU job is the one a 1-GPU job under torchrun executes
        self.dist = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.dist else 1
        self.rank = dist.get_rank(group) if self.dist else 0
        if noise == "reference" and self.world > 1:
            raise ValueError("noise='reference' follows one process's global generator; use 'philox' when sharded")
        self.noise = noise
        self.nfes = 0  # denoise calls (candidates), as search_algorithm.py:72 counts them
        self.device = sampler.model.device
        self.best_image: Optional[torch.Tensor] = None  # denoised image of the search's best candidate
        self._best_owner = -1
        self._ref_pending: Optional[Tuple[torch.Tensor, torch.Tensor]] = None

    def reserve(self, n_candidates: int, noise_shape) -> None:
        """Size the native UNet for this rank's shard of a round up front (weights are packed
        once per capacity; a later, larger round would otherwise re-create the handle)."""
        _, nl = self.shard(n_candidates)
        native = getattr(self.sampler, "_native", None)  # (sampler stand-ins in the CPU tests have none)
        if native is not None:
            native(nl * int(noise_shape[0]))  # the same batch sampler.run sizes the handle with

    def shard(self, n: int) -> Tuple[int, int]:
        if n % self.world:
            raise ValueError(f"{n} candidates do not split evenly over {self.world} ranks")
        nl = n // self.world
        return self.rank * nl, nl

    def candidate_noise(self, round_id: int, g0: int, count: int, shape, pivot: Optional[torch.Tensor] = None,
                        scale: float = 1.0) -> torch.Tensor:
        """x_T of candidates g0..g0+count-1 of a round (a pure function of their global index)."""
        out = torch.empty((count * shape[0],) + tuple(shape[1:]), dtype=torch.float32, device=self.device)
        sid = (_STREAM_PERTURB if pivot is not None else _STREAM_XT) + round_id
        if pivot is not None:
            pivot = pivot.to(self.device, torch.float32).contiguous()
        rt.noise(out, count, self.seed, sid, cand_offset=g0, pivot=pivot, scale=scale)
        return out

    def initial_noise(self, shape) -> torch.Tensor:
        """The initial pivot of zero-order / path search: Philox of the engine seed, so every
        rank holds the same pivot whatever its own torch generator state."""
        out = torch.empty(tuple(shape), dtype=torch.float32, device=self.device)
        rt.noise(out, 1, self.seed, _STREAM_INIT, cand_offset=0)
        return out

    def run_round(self, round_id: int, n: int, shape, pivot: Optional[torch.Tensor] = None, scale: float = 1.0,
                  labels: Optional[torch.Tensor] = None, kind: Optional[str] = None) -> RoundResult:
        g0, nl = self.shard(n)
        per = int(torch.Size(shape[1:]).numel()) * shape[0]
        lab = None
        if labels is not None:
            lab = labels.to(self.device).flatten().repeat(nl)
        if self.noise == "reference":
            kind = kind or ("random" if pivot is None else "path")
            x_cpu, z_cpu = ReferenceNoise(self.sampler.T).round(kind, n, shape, pivot, scale)
            self._ref_pending = (x_cpu, z_cpu)
            x = x_cpu.to(self.device, copy=True).contiguous()  # x_cpu stays the drawn x_T
            self.sampler.run(x, labels=lab, noise=z_cpu, graph=self.graph)
        else:
            x = self.candidate_noise(round_id, g0, nl, shape, pivot, scale)
            self.sampler.run(x, labels=lab, seed=(self.seed * 1000003 + round_id) & ((1 << 62) - 1),
                             noise_offset=g0 * per, graph=self.graph)
        local = self.verifier.score_batch(x, nl)
        self.nfes += n
        if self.dist:
            parts = [torch.empty_like(local) for _ in range(self.world)]
            dist.all_gather(parts, local.contiguous(), group=self.group)  # the round's one collective
            scores = torch.cat(parts)
        else:
            scores = local
        sc = scores.cpu()
        best, best_score = strict_argmax(sc)
        return RoundResult(scores=sc, best_index=best, best_score=best_score, local_images=x, g0=g0)

    def _noise_of(self, r: RoundResult, round_id: int, shape, pivot=None, scale: float = 1.0) -> torch.Tensor:
        """x_T of the round's best candidate (regenerated from its global index; parity mode:
        the drawn tensor)."""
        if self.noise == "reference":
            b = shape[0]
            return self._ref_pending[0][r.best_index * b:(r.best_index + 1) * b].to(self.device).clone()
        return self.candidate_noise(round_id, r.best_index, 1, shape, pivot=pivot, scale=scale)

    def _keep_best_image(self, r: RoundResult, shape) -> None:
        """The owner rank of a new best candidate keeps its denoised image (no collective)."""
        b = shape[0]
        nl = r.local_images.shape[0] // b
        owner = r.best_index // nl
        self._best_owner = owner
        if owner == self.rank:
            i = r.best_index - r.g0
            self.best_image = r.local_images[i * b:(i + 1) * b].clone()
        else:
            self.best_image = None

    def _publish_best_image(self, shape) -> None:
        """One broadcast from the owner at the end of the search (under a process group)."""
        if self.dist and self._best_owner >= 0:
            if self.best_image is None:
                self.best_image = torch.empty(tuple(shape), dtype=torch.float32, device=self.device)
            # the owner is a rank of self.group; broadcast's src is a global rank
            src = self._best_owner if self.group is None else dist.get_global_rank(self.group, self._best_owner)
            dist.broadcast(self.best_image, src=src, group=self.group)

    # --- the three searches, batched
    def random_search(self, n_candidates: int, noise_shape) -> Tuple[Optional[torch.Tensor], float, Dict[str, Any]]:
        self.best_image, self._best_owner = None, -1
        self.reserve(n_candidates, noise_shape)
        r = self.run_round(0, n_candidates, noise_shape, kind="random")
        best_noise = None  # search_algorithm.py:60 (no candidate beat -inf)
        if r.best_index >= 0:
            best_noise = self._noise_of(r, 0, noise_shape)
            self._keep_best_image(r, noise_shape)
        self._publish_best_image(noise_shape)
        return best_noise, r.best_score, {"scores": r.scores.tolist(), "best_index": r.best_index}

    def zero_order_search(self, initial_noise: torch.Tensor, n_neighbors: int, lambda_radius: float,
                          n_iterations: int, labels=None):
        shape = tuple(initial_noise.shape)
        self.best_image, self._best_owner = None, -1
        self.reserve(n_neighbors, shape)
        pivot = initial_noise.to(self.device, torch.float32).contiguous()
        best_noise, best_score = pivot.clone(), float("-inf")
        hist = {"scores": [], "candidates_per_iter": [], "best_index": []}
        for it in range(n_iterations):
            r = self.run_round(1 + it, n_neighbors, shape, pivot=pivot, scale=1 - lambda_radius, labels=labels,
                               kind="zero_order")
            hist["scores"].append(r.scores.tolist())
            hist["candidates_per_iter"].append(n_neighbors)
            hist["best_index"].append(r.best_index)
            if r.best_score > best_score:  # search_algorithm.py:193-196
                best_score = r.best_score
                cand = self._noise_of(r, 1 + it, shape, pivot=pivot, scale=1 - lambda_radius)
                best_noise, pivot = cand.clone(), cand.clone()
                self._keep_best_image(r, shape)
        self._publish_best_image(shape)
        return best_noise, best_score, hist

    def path_search(self, initial_noise: torch.Tensor, n_paths: int, noise_scale: float, injection_step: int = 400,
                    labels=None):
        shape = tuple(initial_noise.shape)
        self.best_image, self._best_owner = None, -1
        self.reserve(n_paths, shape)
        pivot = initial_noise.to(self.device, torch.float32).contiguous()
        r = self.run_round(0, n_paths, shape, pivot=pivot, scale=noise_scale, labels=labels, kind="path")
        best = pivot.clone()  # search_algorithm.py:292 (kept when no path beats -inf)
        if r.best_index >= 0:
            best = self._noise_of(r, 0, shape, pivot=pivot, scale=noise_scale)
            self._keep_best_image(r, shape)
        self._publish_best_image(shape)
        return best, r.best_score, {"scores": r.scores.tolist(), "injection_points": [injection_step] * n_paths,
                                    "best_index": r.best_index}


# --------------------------------------------------------------------------- reference API
def _iter(n, verbose, desc):
    if verbose:
        try:
            from tqdm import tqdm

            return tqdm(range(n), desc=desc, leave=False)
        except ImportError:  # pragma: no cover
            pass
    return range(n)


def _engine(sampler, verifier_fn, seed, reference_rng):
    if sampler is None:
        raise ValueError("batched=True needs sampler= (an itsd GaussianDiffusionSampler)")
    return SearchEngine(sampler, verifier_fn, seed=seed, noise="reference" if reference_rng else "philox")


class RandomSearch:
    """``search_algorithm.py:18-87``."""

    def __init__(self, n_candidates: int = 4):
        self.n_candidates = n_candidates
        self.nfes = 0

    def search(self, noise_shape: Tuple[int, ...], denoise_fn: Callable, verifier_fn: Callable,
               device: str = "cuda", verbose: bool = True, batched: bool = False, sampler=None, seed: int = 0,
               reference_rng: bool = False, **kwargs):
        if batched:
            eng = _engine(sampler, verifier_fn, seed, reference_rng)
            best_noise, best_score, _ = eng.random_search(self.n_candidates, noise_shape)
            self.nfes += self.n_candidates
            return best_noise, best_score
        best_noise, best_score = None, float("-inf")
        for i in _iter(self.n_candidates, verbose, f"Random Search ({self.n_candidates} candidates)"):
            noise = torch.randn(noise_shape, device=device)
            with torch.no_grad():
                denoised = denoise_fn(noise, show_progress=(i == 0), **kwargs)
                self.nfes += 1
            score = verifier_fn(denoised, **kwargs)
            if score > best_score:
                best_score, best_noise = score, noise.clone()
        return best_noise, best_score

    def reset_nfes(self):
        self.nfes = 0


class ZeroOrderSearch:
    """``search_algorithm.py:90-235``."""

    def __init__(self, n_neighbors: int = 4, lambda_radius: float = 0.95, n_iterations: int = 10,
                 verbose: bool = False):
        self.n_neighbors = n_neighbors
        self.lambda_radius = lambda_radius
        self.n_iterations = n_iterations
        self.verbose = verbose
        self.nfes = 0

    def search(self, initial_noise: torch.Tensor, denoise_fn: Callable, verifier_fn: Callable, device: str = "cuda",
               verbose: Optional[bool] = None, batched: bool = False, sampler=None, seed: int = 0,
               reference_rng: bool = False, **kwargs):
        if batched:
            eng = _engine(sampler, verifier_fn, seed, reference_rng)
            out = eng.zero_order_search(initial_noise, self.n_neighbors, self.lambda_radius, self.n_iterations)
            self.nfes += self.n_neighbors * self.n_iterations
            return out
        current = initial_noise.clone()
        best_noise, best_score = initial_noise.clone(), float("-inf")
        history = {"scores": [], "candidates_per_iter": []}
        for _ in range(self.n_iterations):
            neighbors = self._sample_neighbors(current, device)
            its, bc, bcs = [], None, float("-inf")
            for idx, nb in enumerate(neighbors):
                with torch.no_grad():
                    den = denoise_fn(nb, show_progress=(idx == 0), **kwargs)
                    self.nfes += 1
                s = verifier_fn(den, **kwargs)
                its.append(s)
                if s > bcs:
                    bcs, bc = s, nb.clone()
            history["scores"].append(its)
            history["candidates_per_iter"].append(len(neighbors))
            if bcs > best_score:
                best_score, best_noise, current = bcs, bc.clone(), bc.clone()
        return best_noise, best_score, history

    def _sample_neighbors(self, pivot: torch.Tensor, device: str) -> List[torch.Tensor]:
        return [pivot + torch.randn_like(pivot) * (1 - self.lambda_radius) for _ in range(self.n_neighbors)]

    def reset_nfes(self):
        self.nfes = 0


class PathSearch:
    """``search_algorithm.py:238-340`` (the reference's injection is a placeholder:
    each path denoises ``initial + noise_scale * randn`` from T)."""

    def __init__(self, n_paths: int = 4, injection_step: int = 400, noise_scale: float = 0.1, verbose: bool = False):
        self.n_paths = n_paths
        self.injection_step = injection_step
        self.noise_scale = noise_scale
        self.verbose = verbose
        self.nfes = 0

    def search(self, initial_noise: torch.Tensor, denoise_fn: Callable, verifier_fn: Callable, timesteps: int = 1000,
               device: str = "cuda", verbose: Optional[bool] = None, batched: bool = False, sampler=None,
               seed: int = 0, reference_rng: bool = False, **kwargs):
        if batched:
            eng = _engine(sampler, verifier_fn, seed, reference_rng)
            out = eng.path_search(initial_noise, self.n_paths, self.noise_scale, self.injection_step)
            self.nfes += self.n_paths
            return out
        best_noise, best_score = initial_noise.clone(), float("-inf")
        history = {"scores": [], "injection_points": []}
        for path_idx in range(self.n_paths):
            pert = initial_noise + torch.randn_like(initial_noise) * self.noise_scale
            with torch.no_grad():
                den = denoise_fn(pert, show_progress=(path_idx == 0), **kwargs)
                self.nfes += 1
            s = verifier_fn(den, **kwargs)
            history["scores"].append(s)
            history["injection_points"].append(self.injection_step)
            if s > best_score:
                best_score, best_noise = s, pert.clone()
        return best_noise, best_score, history

    def reset_nfes(self):
        self.nfes = 0
