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
    dev = torch.device(cfg.get("device") or "cuda")
    if dev.type != "cuda":
        raise ValueError("itsd samples on the GPU only; set device: cuda")
    if dev.index is None:
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", torch.cuda.current_device())))
    return dev


def _weights(cfg: Dict[str, Any], net, dir_key: str) -> str:
    mode = cfg.get("weights")
    path = _checkpoint_path(cfg, dir_key)
    if mode == "random" or (mode is None and path is None):
        return "random"  # the facade already holds the seeded synthetic recipe
    if path is None:
        raise ValueError("weights: checkpoint needs test_load_weight (+ save_weight_dir/save_dir) or checkpoint_path")
    net.load_state_dict(load_checkpoint_state_dict(path))
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


def _search(cfg: Dict[str, Any], sampler, img_size: int, labels: Optional[torch.Tensor]) -> Optional[Dict[str, Any]]:
    s = cfg.get("search") or {}
    algo = (s.get("algorithm") or "none").lower()
    if algo == "none":
        return None
    from .search import SearchEngine
    from .verifier import AestheticPredictor, OracleVerifier, SelfSupervisedVerifier

    ver = {"oracle": OracleVerifier, "selfsup": SelfSupervisedVerifier,
           "aesthetic": AestheticPredictor}[(s.get("verifier") or "oracle").lower()]()
    eng = SearchEngine(sampler, ver, seed=int(cfg.get("seed") or 0))
    shape = (int(s.get("batch_per_candidate") or 1), 3, img_size, img_size)
    lab = None if labels is None else labels[:shape[0]]
    if algo == "random":
        if lab is not None:
            raise ValueError("search.algorithm random is unconditional (search_algorithm.py:33-83)")
        best, score, hist = eng.random_search(int(s.get("n_candidates") or 4), shape)
    else:
        init = torch.randn(shape, device=sampler.model.device)
        if algo == "zero_order":
            best, score, hist = eng.zero_order_search(init, int(s.get("n_neighbors") or 4),
                                                      float(s.get("lambda_radius", 0.95)),
                                                      int(s.get("n_iterations") or 10), labels=lab)
        elif algo == "path":
            best, score, hist = eng.path_search(init, int(s.get("n_paths") or 4), float(s.get("noise_scale", 0.1)),
                                                int(s.get("injection_step") or 400), labels=lab)
        else:
            raise ValueError(f"unknown search.algorithm '{algo}'")
    x = best.clone()
    sampler.run(x, labels=lab, seed=int(cfg.get("seed") or 0) + 7)
    out = {"algorithm": algo, "best_score": score, "nfes": eng.nfes, "history": hist}
    if eng.rank == 0:
        d = cfg.get("sampled_dir") or "./SampledImgs/"
        save_image(x * 0.5 + 0.5, os.path.join(d, s.get("bestImgName") or "SearchBestImgs.png"), nrow=cfg.get("nrow", 8))
        with open(os.path.join(d, (s.get("bestImgName") or "SearchBestImgs.png").rsplit(".", 1)[0] + ".json"), "w") as fh:
            json.dump(out, fh)
    out["best_image"] = x
    return out


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
        d = cfg["sampled_dir"]
        os.makedirs(d, exist_ok=True)
        save_image(torch.clamp(noisy * 0.5 + 0.5, 0, 1), os.path.join(d, cfg["sampledNoisyImgName"]), nrow=cfg["nrow"])
        imgs = sampler(noisy) * 0.5 + 0.5
        save_image(imgs, os.path.join(d, cfg["sampledImgName"]), nrow=cfg["nrow"])
        res = {"noisy": noisy, "sampled": imgs}
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
        d = cfg["sampled_dir"]
        os.makedirs(d, exist_ok=True)
        save_image(torch.clamp(noisy * 0.5 + 0.5, 0, 1), os.path.join(d, cfg["sampledNoisyImgName"]), nrow=cfg["nrow"])
        imgs = sampler(noisy, labels) * 0.5 + 0.5
        save_image(imgs, os.path.join(d, cfg["sampledImgName"]), nrow=cfg["nrow"])
        res = {"noisy": noisy, "sampled": imgs, "labels": labels}
        res["search"] = _search(cfg, sampler, img, labels)
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
    return eval_condition(cfg) if condition else eval(cfg)


def main(argv: Optional[Sequence[str]] = None, condition: bool = False, default_name: str = "config") -> Dict[str, Any]:
    path, overrides = parse_argv(sys.argv[1:] if argv is None else argv, default_name)
    cfg = load_config(path, overrides)
    print("=" * 80)
    for k, v in sorted(cfg.items()):
        print(f"  {k}: {v}")
    print("=" * 80)
    return run(cfg, condition)
