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
   the same argmax (strict '>' scan order = lowest global index on ties,
   ``search_algorithm.py:79``). The winner's noise is regenerated locally from its
   global index, so no noise ever crosses xGMI.
"""
from __future__ import annotations

import dataclasses
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import runtime as rt

_STREAM_XT = 0xF0000000      # Philox stream ids (the sampler uses stream id = t < T)
_STREAM_PERTURB = 0xE0000000


# --------------------------------------------------------------------------- engine
@dataclasses.dataclass
class RoundResult:
    scores: torch.Tensor          # [N] fp64 (all candidates, every rank)
    best_index: int               # global index of the round's best candidate
    best_score: float
    local_images: torch.Tensor    # this rank's denoised candidates [n_local*B,3,H,W]


class SearchEngine:
    """Batched, sharded search rounds over a sampler + native verifier."""

    def __init__(self, sampler, verifier, seed: int = 0, group=None, graph: bool = True):
        if not hasattr(verifier, "kind"):
            raise TypeError("SearchEngine needs an itsd verifier (OracleVerifier / SelfSupervisedVerifier / "
                            "AestheticPredictor); wrap custom scorers in the sequential API")
        self.sampler = sampler
        self.verifier = verifier
        self.seed = int(seed)
        self.group = group
        self.graph = graph
        self.world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        self.nfes = 0  # denoise calls (candidates), as search_algorithm.py:72 counts them
        self.device = sampler.model.device

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

    def run_round(self, round_id: int, n: int, shape, pivot: Optional[torch.Tensor] = None, scale: float = 1.0,
                  labels: Optional[torch.Tensor] = None) -> RoundResult:
        g0, nl = self.shard(n)
        x = self.candidate_noise(round_id, g0, nl, shape, pivot, scale)
        per = x[0:shape[0]].numel()
        lab = None
        if labels is not None:
            lab = labels.to(self.device).flatten().repeat(nl)
        self.sampler.run(x, labels=lab, seed=(self.seed * 1000003 + round_id) & ((1 << 62) - 1),
                         noise_offset=g0 * per, graph=self.graph)
        local = self.verifier.score_batch(x, nl)
        self.nfes += n
        if self.world > 1:
            parts = [torch.empty_like(local) for _ in range(self.world)]
            dist.all_gather(parts, local.contiguous(), group=self.group)  # the round's one collective
            scores = torch.cat(parts)
        else:
            scores = local
        sc = scores.cpu()
        best = int(torch.argmax(sc).item())  # first occurrence of the max (strict '>')
        if torch.isnan(sc).all():
            best = 0
        return RoundResult(scores=sc, best_index=best, best_score=float(sc[best]), local_images=x)

    # --- the three searches, batched
    def random_search(self, n_candidates: int, noise_shape) -> Tuple[torch.Tensor, float, Dict[str, Any]]:
        r = self.run_round(0, n_candidates, noise_shape)
        best_noise = self.candidate_noise(0, r.best_index, 1, noise_shape)
        return best_noise, r.best_score, {"scores": r.scores.tolist(), "best_index": r.best_index}

    def zero_order_search(self, initial_noise: torch.Tensor, n_neighbors: int, lambda_radius: float,
                          n_iterations: int, labels=None):
        shape = tuple(initial_noise.shape)
        pivot = initial_noise.to(self.device, torch.float32).contiguous()
        best_noise, best_score = pivot.clone(), float("-inf")
        hist = {"scores": [], "candidates_per_iter": [], "best_index": []}
        for it in range(n_iterations):
            r = self.run_round(1 + it, n_neighbors, shape, pivot=pivot, scale=1 - lambda_radius, labels=labels)
            hist["scores"].append(r.scores.tolist())
            hist["candidates_per_iter"].append(n_neighbors)
            hist["best_index"].append(r.best_index)
            if r.best_score > best_score:  # search_algorithm.py:193-196
                best_score = r.best_score
                cand = self.candidate_noise(1 + it, r.best_index, 1, shape, pivot=pivot, scale=1 - lambda_radius)
                best_noise, pivot = cand.clone(), cand.clone()
        return best_noise, best_score, hist

    def path_search(self, initial_noise: torch.Tensor, n_paths: int, noise_scale: float, injection_step: int = 400,
                    labels=None):
        shape = tuple(initial_noise.shape)
        pivot = initial_noise.to(self.device, torch.float32).contiguous()
        r = self.run_round(0, n_paths, shape, pivot=pivot, scale=noise_scale, labels=labels)
        best = self.candidate_noise(0, r.best_index, 1, shape, pivot=pivot, scale=noise_scale)
        return best, r.best_score, {"scores": r.scores.tolist(), "injection_points": [injection_step] * n_paths}


# --------------------------------------------------------------------------- reference API
def _iter(n, verbose, desc):
    if verbose:
        try:
            from tqdm import tqdm

            return tqdm(range(n), desc=desc, leave=False)
        except ImportError:  # pragma: no cover
            pass
    return range(n)


class RandomSearch:
    """``search_algorithm.py:18-87``."""

    def __init__(self, n_candidates: int = 4):
        self.n_candidates = n_candidates
        self.nfes = 0

    def search(self, noise_shape: Tuple[int, ...], denoise_fn: Callable, verifier_fn: Callable,
               device: str = "cuda", verbose: bool = True, batched: bool = False, sampler=None, seed: int = 0,
               **kwargs):
        if batched:
            eng = SearchEngine(sampler, verifier_fn, seed=seed)
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
               verbose: Optional[bool] = None, batched: bool = False, sampler=None, seed: int = 0, **kwargs):
        if batched:
            eng = SearchEngine(sampler, verifier_fn, seed=seed)
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
               seed: int = 0, **kwargs):
        if batched:
            eng = SearchEngine(sampler, verifier_fn, seed=seed)
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
