"""DDPM eval entry point (drop-in for the reference's ``Main.py`` with ``state: eval``).

    python Main.py                                   # config/config.yaml
    python Main.py --config-name inference_config checkpoint_path=ckpt.pt
    python Main.py weights=random batch_size=16 inference_T=50 precision=bf16
    torchrun --nproc-per-node 8 Main.py search.algorithm=random search.n_candidates=1024
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from itsd.entry import load_config, main, run  # noqa: E402,F401

if __name__ == "__main__":
    main(condition=False, default_name="config")
