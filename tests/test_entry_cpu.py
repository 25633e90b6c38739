"""Host logic of the eval entry points (itsd/entry.py <- Main.py, Train.py:808-843,
MainCondition.py, TrainCondition.py:118-151): config surface, checkpoint loading, label
layout, image grids. No GPU compute here."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT
from itsd import entry as E
from itsd.arch import ARCH_TINY
from itsd.weights import synthetic_state_dict


def test_default_configs_load_with_reference_keys():
    c = E.load_config(os.path.join(ROOT, "config", "config.yaml"))
    for k in ("T", "inference_T", "beta_1", "beta_T", "channel", "channel_mult", "attn", "num_res_blocks", "dropout",
              "img_size", "batch_size", "device", "save_weight_dir", "test_load_weight", "sampled_dir",
              "sampledNoisyImgName", "sampledImgName", "nrow"):
        assert k in c, k
    assert c["beta_1"] == 1e-4 and isinstance(c["beta_1"], float)
    assert c["inference_T"] is None
    ci = E.load_config(None, config_name="inference_config")
    assert "checkpoint_path" in ci
    cc = E.load_config(None, config_name="condition_config")
    assert cc["w"] == 1.8 and cc["channel_mult"] == [1, 4, 8, 8, 4, 2] and cc["T"] == 3000


def test_hydra_style_overrides_and_legacy_model_config():
    c = E.load_config({"T": 1000, "model_config": {"T": 5, "epoch": 3}, "x": "None", "y": "true", "z": "FALSE"},
                      ["batch_size=16", "channel_mult=[1,2]", "search.algorithm=random", "+new=null", "beta_T=2e-2"])
    assert c["T"] == 1000 and c["epoch"] == 3  # top level wins (Main.py:44-45)
    assert c["x"] is None and c["y"] is True and c["z"] is False  # Main.py:54-62
    assert c["batch_size"] == 16 and c["channel_mult"] == [1, 2] and c["new"] is None
    assert c["search"]["algorithm"] == "random" and c["beta_T"] == 0.02
    p, ov = E.parse_argv(["--config-name", "inference_config", "T=5"], "config")
    assert p.endswith(os.path.join("config", "inference_config.yaml")) and ov == ["T=5"]
    with pytest.raises(ValueError):
        E.load_config({}, ["novalue"])


def _ref_labels(batch_size):
    # the reference loop, TrainCondition.py:122-130
    step = int(batch_size // 10)
    out, k = [], 0
    for i in range(1, batch_size + 1):
        out.append(k)
        if i % step == 0:
            if k < 10 - 1:
                k += 1
    return [v + 1 for v in out]


@pytest.mark.parametrize("b", [10, 25, 64, 80, 256])
def test_cfg_eval_labels(b):
    assert E.cfg_eval_labels(b).tolist() == _ref_labels(b)


def test_cfg_eval_labels_small_batch_rejected():
    with pytest.raises(ValueError):
        E.cfg_eval_labels(9)


def test_make_grid_layout():
    x = torch.arange(5 * 3 * 4 * 4, dtype=torch.float32).reshape(5, 3, 4, 4) / 240.0
    g = E.make_grid(x, nrow=2, padding=2)
    # xmaps = 2, ymaps = 3, each cell (4+2), plus one trailing pad
    assert g.shape == (3, 3 * 6 + 2, 2 * 6 + 2)
    for k in range(5):
        y, xx = divmod(k, 2)
        assert torch.equal(g[:, y * 6 + 2:y * 6 + 6, xx * 6 + 2:xx * 6 + 6], x[k])
    assert g[:, 14:, 8:].abs().sum() == 0  # empty 6th cell stays pad_value
    assert torch.equal(E.make_grid(x[:1]), x[0])  # one image: no padding
    u8 = E.grid_to_uint8(torch.tensor([[[0.0, 0.5, 1.0, 1.2, -0.1, 0.998]]]))
    assert u8[..., 0].tolist() == [[0, 128, 255, 255, 0, 254]]


def test_save_image_png_roundtrip(tmp_path):
    from PIL import Image

    x = torch.rand(10, 3, 8, 8)
    p = str(tmp_path / "g.png")
    E.save_image(x, p, nrow=4)
    arr = np.asarray(Image.open(p))
    assert arr.shape == (3 * 10 + 2, 4 * 10 + 2, 3)
    np.testing.assert_array_equal(arr, E.grid_to_uint8(E.make_grid(x, nrow=4)))


def test_checkpoint_loading_strips_module_prefix(tmp_path):
    sd = synthetic_state_dict(ARCH_TINY, 3)
    p1, p2 = str(tmp_path / "a.pt"), str(tmp_path / "b.pt")
    torch.save({"module." + k: v for k, v in sd.items()}, p1)  # DataParallel checkpoint
    torch.save({"state_dict": sd}, p2)
    for p in (p1, p2):
        got = E.load_checkpoint_state_dict(p)
        assert list(got) == list(sd)
        assert all(torch.equal(got[k], sd[k]) for k in sd)
    with pytest.raises(FileNotFoundError):
        E.load_checkpoint_state_dict(str(tmp_path / "missing.pt"))
    assert E._checkpoint_path({"save_weight_dir": "d", "test_load_weight": "c.pt"}, "save_weight_dir") == \
        os.path.join("d", "c.pt")
    assert E._checkpoint_path({"checkpoint_path": "x.pt", "test_load_weight": "c.pt"}, "save_weight_dir") == "x.pt"


def test_train_state_and_cpu_device_rejected():
    with pytest.raises(NotImplementedError):
        E.run({"state": "train"})
    with pytest.raises(ValueError):
        E._device({"device": "cpu"})


def test_png_grid_geometry_matches_reference_images(tmp_path):
    """The grids save_image writes have the geometry of the reference's own PNGs
    (SampledImgs/*.png, tests/golden/png_grids.json by tools/gen_golden_png.py): 8 x 8 and 8 x 10
    grids of 32-px images -> 274 x 274 and 274 x 342, 8-bit RGB (PNG colour type 2), and the
    2-pixel separators are 0 as in the reference files (padding_max 0 there). Pixel values are
    unpinned: the reference ships no seeds or weights for its images."""
    import json
    import struct

    from PIL import Image

    with open(os.path.join(ROOT, "tests", "golden", "png_grids.json")) as fh:
        gold = json.load(fh)
    for name, g in gold.items():
        n = g["rows"] * g["cols"]
        x = torch.rand(n, 3, 32, 32) * 0.8 + 0.1  # strictly inside (0, 1): no pixel is 0
        p = str(tmp_path / name)
        E.save_image(x, p, nrow=8)
        with open(p, "rb") as fh:
            head = fh.read(33)
        w, h = struct.unpack(">II", head[16:24])
        assert (w, h, head[24], head[25]) == (g["width"], g["height"], g["bit_depth"], g["color_type"]), name
        arr = np.asarray(Image.open(p))
        pad = [r for r in range(h) if r % 34 in (0, 1)]
        padc = [c for c in range(w) if c % 34 in (0, 1)]
        assert max(arr[pad].max(), arr[:, padc].max()) == g["padding_max"] == 0
        inner = np.delete(np.delete(arr, pad, axis=0), padc, axis=1)
        assert inner.min() > 0  # every non-separator pixel belongs to an image
