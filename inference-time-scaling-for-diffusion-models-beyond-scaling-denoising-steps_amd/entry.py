"""Eval entry points with the reference's configuration surface.

* ``eval(cfg)``            <- ``Diffusion/Train.py:808-843`` (``Main.py`` with ``state: eval``)
* ``eval_condition(cfg)``  <- ``DiffusionFreeGuidence/TrainCondition.py:118-151`` (``MainCondition.py``)
* ``load_config``          <- ``Main.py:31-70`` (Hydra ``config_name`` + ``key=value`` overrides,
  legacy ``model_config.*`` flattening, "none"/"null"/"true"/"false" strings)
* ``load_checkpoint_state_dict`` <- ``abstract_metrics_from_pretrained_ddpm.py:126-160``
  (``{"state_dict": ...}`` wrappers, DataParallel ``module.`` prefix)
* ``save_image`` / ``make_grid``: torchvision's grid writer as the reference calls it
  (``save_image(x, path, nrow=cfg["nrow"])``, padding 2, pad value 0, ``x*255+0.5`` clamped
  to uint8, PNG through PIL). torchvision is absent here, so its layout is restated from its
  published algorithm (pixel parity "unpinned" against torchvision itself).

Keys beyond the reference (all optional):

* ``weights``: ``"checkpoint"`` (default when a checkpoint path is set) or ``"random"``
  (the seeded synthetic recipe of ``itsd.weights``; the reference cannot run without a
  checkpoint, and none can be fetched offline);
* ``precision``: ``"fp32"`` (parity, default) or ``"bf16"`` (throughput);
* ``seed``: torch seed for the initial noise and the sampler's Philox streams;
* ``search``: a block selecting a search over initial noise (``search/search_algorithm.py``)
  run batched (and sharded over ranks when launched with torchrun) by ``itsd.search.SearchEngine``::

      search:
        algorithm: random        # random | zero_order | path | none
        n_candidates: 256        # random
        n_neighbors: 4           # zero_order
        lambda_radius: 0.95
        n_iterations: 10
        n_paths: 4               # path
        injection_step: 400
        noise_scale: 0.1
        verifier: oracle         # oracle | selfsup | aesthetic
        bestImgName: SearchBestImgs.png

There is no training entry: ``state: train`` raises (training is out of scope).
"""
from __future__ import annotations

import copy
import json
import math
import os
import sys
from collections import OrderedDict
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch
import yaml

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIG_DIR = os.path.join(REPO_ROOT, "config")


# ----------------------------------------------------------------------------- config
def _coerce(value: str) -> Any:
    """Hydra-style override value: YAML scalar/list syntax (``[1,2]``, ``1e-4``, ``null``)."""
    try:
        v = yaml.safe_load(value)
    except yaml.YAMLError:
        return value
    if isinstance(v, str):
        try:  # YAML 1.1 reads "1e-4" as a string; Hydra/OmegaConf read it as a float
            return float(v) if any(c in v for c in "eE.") else v
        except ValueError:
            return v
    return v


def _set_nested(d: Dict[str, Any], dotted: str, value: Any) -> None:
    keys = dotted.split(".")
    for k in keys[:-1]:
        if not isinstance(d.get(k), dict):
            d[k] = {}
        d = d[k]
    d[keys[-1]] = value


def _normalise_scalars(d: Dict[str, Any]) -> Dict[str, Any]:
    """``Main.py:54-62``: "none"/"null" -> None, "true"/"false" -> bool (top level);
    also turns YAML-1.1 exponent strings (``1e-4``) into floats as OmegaConf does."""
    for k, v in list(d.items()):
        if isinstance(v, str):
            lv = v.lower()
            if lv in ("none", "null"):
                d[k] = None
            elif lv == "true":
                d[k] = True
            elif lv == "false":
                d[k] = False
            else:
                try:
                    if any(c in v for c in "eE") and not v.isalpha():
                        d[k] = float(v)
                except ValueError:
                    pass
    return d


def load_config(config: Optional[Any] = None, overrides: Sequence[str] = (),
                config_name: str = "config") -> Dict[str, Any]:
    """Configuration dict as ``Main.py:load_config`` produces it.

    ``config``: a dict, a YAML path, or None (``config/<config_name>.yaml`` of this repo).
    ``overrides``: Hydra-style ``key=value`` / ``a.b=value`` / ``+key=value`` strings.
    """
    if config is None:
        config = os.path.join(CONFIG_DIR, config_name + ".yaml")
    if isinstance(config, str):
        with open(config) as fh:
            cfg = yaml.safe_load(fh) or {}
    else:
        cfg = copy.deepcopy(dict(config))
    cfg.pop("hydra", None)
    for ov in overrides:
        if "=" not in ov:
            raise ValueError(f"override '{ov}' is not key=value")
        k, v = ov.split("=", 1)
        k = k.lstrip("+~")
        _set_nested(cfg, k, _coerce(v))
    if isinstance(cfg.get("model_config"), dict):  # Main.py:37-48: top level takes precedence
        nested = cfg.pop("model_config")
        cfg = {**nested, **cfg}
    return _normalise_scalars(cfg)


def parse_argv(argv: Sequence[str], default_name: str) -> Tuple[Optional[str], List[str]]:
    """``--config-name X`` / ``--config-path P`` / ``--config-dir P`` and ``key=value`` args."""
    name, cdir, overrides = default_name, CONFIG_DIR, []
    it = iter(argv)
    for a in it:
        if a in ("--config-name", "-cn"):
            name = next(it)
        elif a.startswith("--config-name="):
            name = a.split("=", 1)[1]
        elif a in ("--config-path", "-cp", "--config-dir", "-cd"):
            cdir = next(it)
        elif a.startswith(("--config-path=", "--config-dir=")):
            cdir = a.split("=", 1)[1]
        else:
            overrides.append(a)
    path = os.path.join(cdir, name if name.endswith(".yaml") else name + ".yaml")
    return path, overrides


# ----------------------------------------------------------------------------- checkpoints
def load_checkpoint_state_dict(path: str) -> "OrderedDict[str, torch.Tensor]":
    """State dict of a reference checkpoint (``torch.save(model.state_dict())``,
    ``Train.py:717``), loaded with ``weights_only=True`` (nothing in the file executes)."""
    if not os.path.exists(path):
        raise FileNotFoundError(f"Checkpoint not found: {path}")
    ck = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(ck, dict) and "state_dict" in ck and isinstance(ck["state_dict"], dict):
        ck = ck["state_dict"]
    if not isinstance(ck, dict):
        raise ValueError("Could not extract state_dict from checkpoint")
    return OrderedDict((k[7:] if k.startswith("module.") else k, v) for k, v in ck.items())


def _checkpoint_path(cfg: Dict[str, Any], dir_key: str) -> Optional[str]:
    if cfg.get("checkpoint_path"):  # inference_config.yaml
        return cfg["checkpoint_path"]
    w = cfg.get("test_load_weight")
    if not w:
        return None
    return os.path.join(cfg.get(dir_key) or "", w)  # Train.py:816-817 / TrainCondition.py:134-135


# ----------------------------------------------------------------------------- images
def make_grid(t: torch.Tensor, nrow: int = 8, padding: int = 2, pad_value: float = 0.0) -> torch.Tensor:
    """torchvision ``make_grid`` (no normalisation): images left-to-right, top-to-bottom,
    ``padding`` pixels of ``pad_value`` around and between them; one image is returned as is."""
    t = t.detach().float().cpu()
    if t.dim() == 2:
        t = t.unsqueeze(0)
    if t.dim() == 3:
        if t.size(0) == 1:
            t = torch.cat((t, t, t), 0)
        t = t.unsqueeze(0)
    if t.dim() == 4 and t.size(1) == 1:
        t = torch.cat((t, t, t), 1)
    if t.size(0) == 1:
        return t.squeeze(0)
    nmaps = t.size(0)
    xmaps = min(nrow, nmaps)
    ymaps = int(math.ceil(float(nmaps) / xmaps))
    height, width = int(t.size(2) + padding), int(t.size(3) + padding)
    grid = t.new_full((t.size(1), height * ymaps + padding, width * xmaps + padding), pad_value)
    k = 0
    for y in range(ymaps):
        for x in range(xmaps):
            if k >= nmaps:
                break
            grid[:, y * height + padding:(y + 1) * height, x * width + padding:(x + 1) * width] = t[k]
            k += 1
    return grid


def grid_to_uint8(grid: torch.Tensor):
    """``save_image``'s quantisation: ``x*255 + 0.5`` clamped to [0,255], truncated to uint8, HWC."""
    return grid.mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to(torch.uint8).numpy()


def save_image(t: torch.Tensor, path: str, nrow: int = 8, padding: int = 2) -> None:
    from PIL import Image

    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    Image.fromarray(grid_to_uint8(make_grid(t, nrow=nrow, padding=padding))).save(path)


# ----------------------------------------------------------------------------- eval
def cfg_eval_labels(batch_size: int) -> torch.Tensor:
    """``TrainCondition.py:122-130``: ``batch_size // 10`` consecutive images per class,
    classes 1..10 (the last class takes the remainder)."""
    step = int(batch_size // 10)
    if step == 0:
        raise ValueError("batch_size must be >= 10 (TrainCondition.py:122 divides by batch_size // 10)")
    labels, k = [], 0
    for i in range(1, batch_size + 1):
        labels.append(k)
        if i % step == 0 and k < 10 - 1:
            k += 1
    return torch.tensor(labels, dtype=torch.long) + 1


def _device(cfg: Dict[str, Any]) -> torch.device:
    """``device`` (``Train.py:811``) and the inference config's ``device_ids`` /
    ``use_multi_gpu`` (``abstract_metrics_from_pretrained_ddpm.py:52-123``). itsd runs one
    process per GPU (torchrun) instead of DataParallel: under torchrun rank r takes
    ``device_ids[LOCAL_RANK]``, else ``cuda:(i + LOCAL_RANK)`` for ``device: cuda:i`` (``cuda``:
    i = 0) -- never one GPU for every rank; one process takes ``device_ids[0]`` / ``cuda:i``."""
    spec = str(cfg.get("device") or "cuda")
    if spec.split(":")[0] != "cuda":
        raise ValueError("itsd samples on the GPU only; set device: cuda")
    ids = cfg.get("device_ids")
    if isinstance(ids, str):
        ids = [int(x) for x in ids.replace("[", "").replace("]", "").split(",") if x.strip()]
    elif ids is not None and not isinstance(ids, (list, tuple)):
        ids = [int(ids)]
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))

    def checked(i: int, key: str) -> torch.device:
        n = torch.cuda.device_count()  # (counting devices does not initialise the GPU)
        if n and not 0 <= i < n:
            raise ValueError(f"config key '{key}' selects cuda:{i} but this process sees {n} GPU(s)"
                             + (f" (LOCAL_RANK {local})" if "LOCAL_RANK" in os.environ else ""))
        return torch.device("cuda", i)

    if ids:
        if world > 1 and local >= len(ids):
            raise ValueError(f"device_ids {list(ids)} has no entry for LOCAL_RANK {local}")
        return checked(int(ids[local if world > 1 else 0]), "device_ids")
    dev = torch.device(spec.split(",")[0])
    if world > 1:  # one GPU per rank: the configured index is the first rank's
        return checked((dev.index or 0) + local, "device")
    if dev.index is None:
        return checked(local if "LOCAL_RANK" in os.environ else torch.cuda.current_device(), "device")
    return checked(dev.index, "device")


def detect_checkpoint_T(state_dict: Dict[str, torch.Tensor]) -> Optional[int]:
    """``abstract_metrics_from_pretrained_ddpm.py:163-188``: the row count of
    ``time_embedding.timembedding.0.weight`` when it exceeds 500, else None.

    For the functional DDPM embedding (``Model.py:38-42``) that tensor is the first Linear,
    [4*ch, ch] = [512, 128] at ch = 128, so the reference "detects T = 512" there; for a
    table embedding (``ModelCondition.py:38``, [T, ch]) it is the table's T."""
    w = state_dict.get("time_embedding.timembedding.0.weight")
    if w is not None and w.dim() == 2 and w.shape[0] > 500:
        return int(w.shape[0])
    return None


def time_table(T: int, d_model: int, checkpoint_T: Optional[int] = None, strategy: str = "interpolate") -> torch.Tensor:
    """The sinusoid table ``reinitialize_time_embedding`` builds
    (``abstract_metrics_from_pretrained_ddpm.py:211-248``): sin/cos interleaved over
    positions 0..T-1; with strategy "interpolate" and checkpoint_T < T the first
    checkpoint_T rows are scaled by checkpoint_T / T."""
    f = torch.exp(-(torch.arange(0, d_model, step=2) / d_model * math.log(10000)))
    pos = torch.arange(T).float()
    e = pos[:, None] * f[None, :]
    e = torch.stack([torch.sin(e), torch.cos(e)], dim=-1).view(T, d_model)
    if strategy == "interpolate" and checkpoint_T is not None and checkpoint_T < T:
        out = e.clone()
        out[:checkpoint_T] = e[:checkpoint_T] * (checkpoint_T / T)
        return out
    return e


def adapt_time_embedding(state_dict: "OrderedDict[str, torch.Tensor]", net, cfg: Dict[str, Any]):
    """T-mismatch handling of ``create_and_load_model`` (``abstract_metrics_from_pretrained_ddpm.py:
    312-337``) for a checkpoint loaded into a model built with ``cfg["T"]``.

    * functional DDPM embedding (itsd ``UNet``): T is not stored in any weight, so nothing is
      replaced and every weight loads as trained. (The reference misreads the [512, 128] Linear
      as a T = 512 table, drops every time_embedding weight and writes a [T, 128] sinusoid into
      that Linear, whose forward then fails on the bias shape; itsd keeps the checkpoint.)
    * table embedding (itsd ``CondUNet``, [T_ckpt, ch]): ``time_embedding_strategy``
      "interpolate" / "reinit" rebuilds the table for T as the reference does and re-initialises
      the embedding MLP (xavier-uniform weights, zero biases; ``:257-266``, seeded by
      ``weight_seed``); "strict" (or no strategy key) raises.
    Returns the (possibly rewritten) state dict."""
    ck_T = detect_checkpoint_T(state_dict)
    T = int(cfg["T"])
    if ck_T is None or ck_T == T:
        return state_dict
    if not net.arch.cfg:
        print(f"Functional time embedding: checkpoint tensor time_embedding.timembedding.0.weight "
              f"{tuple(state_dict['time_embedding.timembedding.0.weight'].shape)} is the first MLP Linear, not a "
              f"T={ck_T} table; T={T} needs no weight surgery (loading the checkpoint unchanged)")
        return state_dict
    strategy = (cfg.get("time_embedding_strategy") or "strict").lower()
    if strategy not in ("interpolate", "reinit"):
        raise ValueError(f"checkpoint time-embedding table has T={ck_T} rows, config T={T}; set "
                         f"time_embedding_strategy: interpolate | reinit to rebuild it")
    if cfg.get("fine_tune_time_embedding"):
        print("fine_tune_time_embedding: ignored (itsd is inference-only)")
    print(f"T mismatch: checkpoint T={ck_T}, config T={T}: rebuilding the time embedding ({strategy})")
    sd = OrderedDict((k, v) for k, v in state_dict.items() if not k.startswith("time_embedding"))
    d_model = int(state_dict["time_embedding.timembedding.0.weight"].shape[1])
    sd["time_embedding.timembedding.0.weight"] = time_table(T, d_model, ck_T, strategy)
    gen = torch.Generator().manual_seed(int(cfg.get("weight_seed") or 0))
    for name in ("time_embedding.timembedding.1", "time_embedding.timembedding.3"):
        w = torch.empty_like(state_dict[name + ".weight"])
        torch.nn.init.xavier_uniform_(w, generator=gen)
        sd[name + ".weight"] = w
        sd[name + ".bias"] = torch.zeros_like(state_dict[name + ".bias"])
    return sd


def _weights(cfg: Dict[str, Any], net, dir_key: str) -> str:
    mode = cfg.get("weights")
    path = _checkpoint_path(cfg, dir_key)
    if mode == "random" or (mode is None and path is None):
        return "random"  # the facade already holds the seeded synthetic recipe
    if path is None:
        raise ValueError("weights: checkpoint needs test_load_weight (+ save_weight_dir/save_dir) or checkpoint_path")
    net.load_state_dict(adapt_time_embedding(load_checkpoint_state_dict(path), net, cfg))
    return path


def build_ddpm(cfg: Dict[str, Any]):
    from .model import UNet

    dev = _device(cfg)
    net = UNet(T=cfg["T"], ch=cfg["channel"], ch_mult=cfg["channel_mult"], attn=cfg["attn"],
               num_res_blocks=cfg["num_res_blocks"], dropout=0.0, img_size=int(cfg.get("img_size") or 32),
               precision=cfg.get("precision") or "fp32", weights="gauss", seed=int(cfg.get("weight_seed") or 0),
               device=dev)
    src = _weights(cfg, net, "save_weight_dir")
    print("model load weight done." if src != "random" else "model: synthetic weights (weights: random).")
    return net.eval()


def build_cfg_model(cfg: Dict[str, Any]):
    from .model import CondUNet

    dev = _device(cfg)
    net = CondUNet(T=cfg["T"], num_labels=int(cfg.get("num_labels") or 10), ch=cfg["channel"],
                   ch_mult=cfg["channel_mult"], num_res_blocks=cfg["num_res_blocks"], dropout=cfg.get("dropout", 0.0),
                   img_size=int(cfg.get("img_size") or 32), precision=cfg.get("precision") or "fp32",
                   weights="gauss", seed=int(cfg.get("weight_seed") or 0), device=dev)
    src = _weights(cfg, net, "save_dir")
    print("model load weight done." if src != "random" else "model: synthetic weights (weights: random).")
    return net.eval()


def _json_safe(v):
    """NaN / +-inf scores as null (strict JSON)."""
    if isinstance(v, float):
        return v if math.isfinite(v) else None
    if isinstance(v, dict):
        return {k: _json_safe(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_json_safe(x) for x in v]
    return v


def _rank_world() -> Tuple[int, int]:
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed.get_rank(), torch.distributed.get_world_size()
    return 0, 1


def _search(cfg: Dict[str, Any], sampler, img_size: int, labels: Optional[torch.Tensor]) -> Optional[Dict[str, Any]]:
    s = cfg.get("search") or {}
    algo = (s.get("algorithm") or "none").lower()
    if algo == "none":
        return None
    from .search import SearchEngine
    from .verifier import AestheticPredictor, OracleVerifier, SelfSupervisedVerifier

    vname = (s.get("verifier") or "oracle").lower()
    ver = {"oracle": OracleVerifier, "selfsup": SelfSupervisedVerifier, "aesthetic": AestheticPredictor}[vname]()
    shape = (int(s.get("batch_per_candidate") or 1), 3, img_size, img_size)
    if vname == "selfsup" and shape[0] < 2:
        # verifier.py:243-246 averages the off-diagonal of the in-batch Gram matrix: one image
        # per candidate has none, every score is NaN and the reference search never picks one
        raise ValueError("search.verifier selfsup needs search.batch_per_candidate >= 2")
    eng = SearchEngine(sampler, ver, seed=int(cfg.get("seed") or 0))
    lab = None if labels is None else labels[:shape[0]]
    if algo == "random":
        if lab is not None:
            raise ValueError("search.algorithm random is unconditional (search_algorithm.py:33-83)")
        best, score, hist = eng.random_search(int(s.get("n_candidates") or 4), shape)
    else:
        init = eng.initial_noise(shape)  # the same pivot on every rank (Philox of the seed)
        if algo == "zero_order":
            best, score, hist = eng.zero_order_search(init, int(s.get("n_neighbors") or 4),
                                                      float(s.get("lambda_radius", 0.95)),
                                                      int(s.get("n_iterations") or 10), labels=lab)
        elif algo == "path":
            best, score, hist = eng.path_search(init, int(s.get("n_paths") or 4), float(s.get("noise_scale", 0.1)),
                                                int(s.get("injection_step") or 400), labels=lab)
        else:
            raise ValueError(f"unknown search.algorithm '{algo}'")
    # the winner's own denoised image: kept by its owner rank during the search and broadcast
    # once at the end -- the exact trajectory that earned best_score (not a re-run)
    x = eng.best_image
    out = {"algorithm": algo, "best_score": score, "nfes": eng.nfes, "history": hist}
    if eng.rank == 0 and x is not None:
        d = _out_dir(cfg)
        name = s.get("bestImgName") or "SearchBestImgs.png"
        save_image(x * 0.5 + 0.5, os.path.join(d, name), nrow=cfg.get("nrow", 8))
        with open(os.path.join(d, name.rsplit(".", 1)[0] + ".json"), "w") as fh:
            json.dump(_json_safe(out), fh)
    out["best_noise"] = best
    out["best_image"] = x
    return out


def _out_dir(cfg: Dict[str, Any]) -> str:
    """``sampled_dir`` (config.yaml) or ``sampled_images_save_dir`` (inference_config.yaml)."""
    d = cfg.get("sampled_dir") or cfg.get("sampled_images_save_dir") or "./SampledImgs/"
    os.makedirs(d, exist_ok=True)
    return d


def _sample_sharded(sampler, noisy: torch.Tensor, labels: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``sampler(noisy[, labels])`` with the batch split over the ranks of a torchrun job:
    rank 0's x_T (and labels) are broadcast, every rank runs its contiguous slice with the
    Philox noise of the slice's global image indices, and the result is gathered --
    bit-identical to the single-process run. One process: a plain sampler call.
    ``noisy`` / ``labels`` are overwritten in place with rank 0's values."""
    rank, world = _rank_world()
    if world == 1 or noisy.shape[0] % world:
        return sampler(noisy) if labels is None else sampler(noisy, labels)
    seed = torch.tensor([int(torch.randint(0, 2 ** 62, (1,)).item())], dtype=torch.int64, device=noisy.device)
    torch.distributed.broadcast(seed, src=0)  # one sampler seed even if the ranks' generators differ
    torch.distributed.broadcast(noisy, src=0)  # the saved noisy grid is what every rank slices
    if labels is not None:
        torch.distributed.broadcast(labels, src=0)
    nl = noisy.shape[0] // world
    per = noisy[0].numel()
    x = noisy[rank * nl:(rank + 1) * nl].clone().contiguous()
    lab = None if labels is None else labels[rank * nl:(rank + 1) * nl]
    sampler.run(x, labels=lab, seed=int(seed.item()), noise_offset=rank * nl * per)
    parts = [torch.empty_like(x) for _ in range(world)]
    torch.distributed.all_gather(parts, x)
    return torch.cat(parts)


def eval(cfg: Dict[str, Any]) -> Dict[str, Any]:  # noqa: A001 (reference name)
    """``Train.py:808-843``: sample ``batch_size`` images with ``inference_T`` (default T)
    steps, save the noisy and the sampled grids; then the optional ``search`` block."""
    from .diffusion import GaussianDiffusionSampler

    if cfg.get("seed") is not None:
        torch.manual_seed(int(cfg["seed"]))
    with torch.no_grad():
        model = build_ddpm(cfg)
        inference_T = cfg.get("inference_T") if cfg.get("inference_T") is not None else cfg["T"]
        if inference_T != cfg["T"]:
            print(f"Using inference T={inference_T} (model was trained with T={cfg['T']})")
        else:
            print(f"Using same T={cfg['T']} for inference")
        sampler = GaussianDiffusionSampler(model, cfg["beta_1"], cfg["beta_T"], inference_T)
        img_size = int(cfg.get("img_size") or 256)
        noisy = torch.randn(size=[cfg["batch_size"], 3, img_size, img_size], device=model.device)
        imgs = _sample_sharded(sampler, noisy) * 0.5 + 0.5
        if _rank_world()[0] == 0:
            d = _out_dir(cfg)
            save_image(torch.clamp(noisy * 0.5 + 0.5, 0, 1), os.path.join(d, cfg["sampledNoisyImgName"]),
                       nrow=cfg["nrow"])
            save_image(imgs, os.path.join(d, cfg["sampledImgName"]), nrow=cfg["nrow"])
        res = {"noisy": noisy, "sampled": imgs, "sampler_seed": sampler.last_seed}
        res["search"] = _search(cfg, sampler, img_size, None)
    return res


def eval_condition(cfg: Dict[str, Any]) -> Dict[str, Any]:
    """``TrainCondition.py:118-151``: class-block labels, guided sampling with weight w."""
    from .diffusion import CondGaussianDiffusionSampler

    if cfg.get("seed") is not None:
        torch.manual_seed(int(cfg["seed"]))
    with torch.no_grad():
        labels = cfg_eval_labels(int(cfg["batch_size"]))
        print("labels: ", labels)
        model = build_cfg_model(cfg)
        labels = labels.to(model.device)
        sampler = CondGaussianDiffusionSampler(model, cfg["beta_1"], cfg["beta_T"], cfg["T"], w=cfg["w"])
        img = int(cfg["img_size"])
        noisy = torch.randn(size=[cfg["batch_size"], 3, img, img], device=model.device)
        imgs = _sample_sharded(sampler, noisy, labels) * 0.5 + 0.5
        if _rank_world()[0] == 0:
            d = _out_dir(cfg)
            save_image(torch.clamp(noisy * 0.5 + 0.5, 0, 1), os.path.join(d, cfg["sampledNoisyImgName"]),
                       nrow=cfg["nrow"])
            save_image(imgs, os.path.join(d, cfg["sampledImgName"]), nrow=cfg["nrow"])
        res = {"noisy": noisy, "sampled": imgs, "labels": labels, "sampler_seed": sampler.last_seed}
        res["search"] = _search(cfg, sampler, img, labels)
    return res


def image_filename(cfg: Dict[str, Any]) -> str:
    """``generate_image_filename`` (``abstract_metrics_from_pretrained_ddpm.py:541-588``) without
    metrics: <checkpoint dir name>_T<T>_bs<batch>_size<img>_<timestamp>."""
    from datetime import datetime

    ck = cfg.get("checkpoint_path") or ""
    name = os.path.basename(os.path.dirname(ck)) if ck else "unknown"
    name = name.replace("Checkpoints/", "").replace("checkpoints/", "") or "unknown"
    parts = [name, f"T{cfg.get('T', 'unknown')}", f"bs{cfg.get('batch_size', 'unknown')}",
             f"size{cfg.get('img_size', 'unknown')}", datetime.now().strftime("%Y%m%d_%H%M%S")]
    return "_".join(str(p) for p in parts).replace("/", "-").replace("\\", "-").replace(":", "-")


def infer(cfg: Dict[str, Any]) -> Dict[str, Any]:
    """Pretrained-checkpoint inference with the ``config/inference_config.yaml`` surface
    (``abstract_metrics_from_pretrained_ddpm.py:649-694``): build the DDPM UNet with
    ``T`` / ``channel`` / ... , load ``checkpoint_path`` with the T-mismatch handling of
    ``adapt_time_embedding``, sample ``batch_size`` images at ``img_size`` with a T-step
    sampler, and write ``sampled_images_save_dir/<generate_image_filename>.png`` and
    ``output_dir/metrics_history.json`` (``save_results``, ``:604-646``).

    The FID / IS / CLIP trajectory every ``metric_interval`` steps needs Inception / CLIP
    weights that are downloaded at run time; they are unavailable offline, so
    ``metric_history`` is empty and the JSON says why."""
    from .diffusion import GaussianDiffusionSampler

    if cfg.get("seed") is not None:
        torch.manual_seed(int(cfg["seed"]))
    with torch.no_grad():
        model = build_ddpm(cfg)
        sampler = GaussianDiffusionSampler(model, cfg["beta_1"], cfg["beta_T"], cfg["T"])
        img = int(cfg.get("img_size") or 256)
        x_T = torch.randn(size=[cfg["batch_size"], 3, img, img], device=model.device)
        sampled = _sample_sharded(sampler, x_T)
        res = {"noisy": x_T, "sampled": sampled * 0.5 + 0.5, "image_path": None}
        if _rank_world()[0] == 0:
            out_dir = cfg.get("output_dir") or "./inference_results"
            os.makedirs(out_dir, exist_ok=True)
            img_dir = cfg.get("sampled_images_save_dir") or os.path.join(out_dir, "sampled_images")
            os.makedirs(img_dir, exist_ok=True)
            path = os.path.join(img_dir, image_filename(cfg) + ".png")
            save_image(res["sampled"], path, nrow=cfg.get("nrow", 8))
            print(f"Sampled images saved to: {path}")
            with open(os.path.join(out_dir, "metrics_history.json"), "w") as fh:
                json.dump({"metric_history": [],
                           "note": "FID/IS/CLIP need downloaded Inception/CLIP weights (unavailable offline)"},
                          fh, indent=2)
            res["image_path"] = path
        res["search"] = _search(cfg, sampler, img, None)
    return res


# ----------------------------------------------------------------------------- CLI
def _maybe_init_dist(cfg: Dict[str, Any]) -> None:
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not torch.distributed.is_initialized():
        dev = _device(cfg)
        torch.cuda.set_device(dev)
        torch.distributed.init_process_group("nccl", device_id=dev)


def run(cfg: Dict[str, Any], condition: bool = False) -> Dict[str, Any]:
    if cfg.get("state", "eval") == "train":
        raise NotImplementedError("itsd is inference-only: training (Train.py:train) is out of scope; use state=eval")
    _maybe_init_dist(cfg)
    if condition:
        return eval_condition(cfg)
    # the inference_config.yaml surface has no sampled_dir / sampledImgName keys
    if "sampledImgName" not in cfg and ("sampled_images_save_dir" in cfg or "output_dir" in cfg):
        return infer(cfg)
    return eval(cfg)


def main(argv: Optional[Sequence[str]] = None, condition: bool = False, default_name: str = "config") -> Dict[str, Any]:
    path, overrides = parse_argv(sys.argv[1:] if argv is None else argv, default_name)
    cfg = load_config(path, overrides)
    print("=" * 80)
    for k, v in sorted(cfg.items()):
        print(f"  {k}: {v}")
    print("=" * 80)
    return run(cfg, condition)
