"""Pretrained-checkpoint inference entry point (drop-in for the reference's
``abstract_metrics_from_pretrained_ddpm.py``, config ``config/inference_config.yaml``).

    python abstract_metrics_from_pretrained_ddpm.py checkpoint_path=ckpt.pt
    python abstract_metrics_from_pretrained_ddpm.py weights=random T=1000 img_size=32 batch_size=16
    torchrun --nproc-per-node 8 abstract_metrics_from_pretrained_ddpm.py ...   (batch split over GPUs)

Samples with the reference's inference keys (T, img_size, time_embedding_strategy,
device_ids, sampled_images_save_dir, output_dir, ...) through itsd.entry.infer; the FID /
IS / CLIP metric trajectory needs downloaded weights and is not computed.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from itsd import entry as _entry  # noqa: E402


def main(argv=None):
    path, overrides = _entry.parse_argv(sys.argv[1:] if argv is None else argv, "inference_config")
    cfg = _entry.load_config(path, overrides)
    if cfg.get("state", "eval") == "train":
        raise NotImplementedError("inference entry point: state must be eval")
    _entry._maybe_init_dist(cfg)
    return _entry.infer(cfg)


if __name__ == "__main__":
    main()
