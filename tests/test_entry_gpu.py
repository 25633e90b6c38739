"""End-to-end eval entry points on the GPU (Main.py / MainCondition.py surface) with tiny
UNets loaded from reference-format checkpoint files.

What these tests pin: the entry's plumbing (config keys, checkpoint loading with the `module.`
prefix, seeds, the x_T draw, the sampler call, the PNG grid layout) against a hand-run of the
same itsd components, i.e. the entry against itself. The numerics underneath are pinned
elsewhere (tests/test_gpu_parity.py vs the reference's fixtures). The PNG bytes are
parity-unpinned: torchvision (the reference's save_image) is not installed here, so the grid is
compared with the repo's own torchvision-compatible make_grid."""
import dataclasses
import os

import numpy as np
import pytest
import torch

from itsd import entry as E
from itsd.arch import ARCH_TINY, ARCH_TINY_CFG
from itsd.diffusion import CondGaussianDiffusionSampler, GaussianDiffusionSampler
from itsd.model import CondUNet, UNet
from itsd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu


def _png(path):
    from PIL import Image

    return np.asarray(Image.open(path))


def test_main_eval_ddpm_from_checkpoint(tmp_path):
    a = ARCH_TINY
    sd = synthetic_state_dict(a, 5)
    ck = tmp_path / "ckpt_0_.pt"
    torch.save({"module." + k: v for k, v in sd.items()}, str(ck))
    cfg = E.load_config(None, [f"save_weight_dir={tmp_path}", "test_load_weight=ckpt_0_.pt", "T=1000",
                               "inference_T=8", "channel=32", "channel_mult=[1,2]", "attn=[1]", "num_res_blocks=1",
                               "batch_size=10", f"sampled_dir={tmp_path}/out", "nrow=4", "seed=3"])
    res = E.run(cfg)
    # same run by hand: seed, model, x_T draw on the device, sampler (its Philox seed from the CPU generator)
    torch.manual_seed(3)
    net = UNet(1000, 32, [1, 2], [1], 1, 0.0).to("cuda:0")
    net.load_state_dict(sd)
    x = torch.randn(10, 3, 32, 32, device="cuda:0")
    assert torch.equal(x, res["noisy"])
    ref = GaussianDiffusionSampler(net, 1e-4, 0.02, 8)(x) * 0.5 + 0.5
    assert torch.equal(ref, res["sampled"])
    img = _png(os.path.join(tmp_path, "out", cfg["sampledImgName"]))
    assert img.shape == (3 * 34 + 2, 4 * 34 + 2, 3)
    np.testing.assert_array_equal(img, E.grid_to_uint8(E.make_grid(ref, nrow=4)))
    noisy = _png(os.path.join(tmp_path, "out", cfg["sampledNoisyImgName"]))
    np.testing.assert_array_equal(noisy, E.grid_to_uint8(E.make_grid(torch.clamp(x * 0.5 + 0.5, 0, 1), nrow=4)))


def test_main_condition_eval_and_search(tmp_path):
    a = dataclasses.replace(ARCH_TINY_CFG, T=6)  # the CFG time table has T rows
    sd = synthetic_state_dict(a, 6)
    torch.save(sd, str(tmp_path / "ckpt_63_.pt"))
    cfg = E.load_config(None, [f"save_dir={tmp_path}", "test_load_weight=ckpt_63_.pt", "T=6", "channel=32",
                               "channel_mult=[1,2]", "num_res_blocks=1", "batch_size=10", f"sampled_dir={tmp_path}",
                               "seed=1", "search.algorithm=zero_order", "search.n_neighbors=3",
                               "search.n_iterations=2"], config_name="condition_config")
    res = E.run(cfg, condition=True)
    assert res["labels"].tolist() == list(range(1, 11))
    torch.manual_seed(1)
    net = CondUNet(6, 10, 32, [1, 2], 1, 0.0).to("cuda:0")
    net.load_state_dict(sd)
    x = torch.randn(10, 3, 32, 32, device="cuda:0")
    ref = CondGaussianDiffusionSampler(net, 1e-4, 0.028, 6, w=1.8)(x, res["labels"]) * 0.5 + 0.5
    assert torch.equal(ref, res["sampled"])
    s = res["search"]
    assert s["algorithm"] == "zero_order" and s["nfes"] == 6 and np.isfinite(s["best_score"])
    assert len(s["history"]["scores"]) == 2
    assert os.path.exists(os.path.join(tmp_path, "SearchBestImgs.png"))
    assert os.path.exists(os.path.join(tmp_path, "SearchBestImgs.json"))


def test_main_eval_random_search_synthetic_weights(tmp_path):
    cfg = E.load_config(None, ["weights=random", "inference_T=5", "channel=32", "channel_mult=[1,2]", "attn=[1]",
                               "num_res_blocks=1", "batch_size=2", f"sampled_dir={tmp_path}",
                               "search.algorithm=random", "search.n_candidates=8", "precision=bf16"])
    res = E.run(cfg)
    s = res["search"]
    assert s["nfes"] == 8 and len(s["history"]["scores"]) == 8
    assert s["best_score"] == max(s["history"]["scores"])
    assert s["best_image"].shape == (1, 3, 32, 32)
