"""Classifier-free-guidance eval entry point (drop-in for the reference's ``MainCondition.py``).

    python MainCondition.py                          # config/condition_config.yaml
    python MainCondition.py test_load_weight=ckpt_63_.pt save_dir=./CheckpointsCondition

``main(model_config)`` accepts a config dict as the reference's does.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from itsd.entry import load_config, run  # noqa: E402
from itsd import entry as _entry  # noqa: E402


def main(model_config=None):
    if model_config is not None:
        return run(load_config(model_config), condition=True)
    return _entry.main(condition=True, default_name="condition_config")


if __name__ == "__main__":
    main()
