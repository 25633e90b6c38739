"""Golden vectors for the two verifier branches off the search hot path, produced by the
reference itself (imported by file path from /root/reference; no source copied):
OracleVerifier(dataset_stats=...).score (search/verifier.py:66, the mean) and
SelfSupervisedVerifier.score(images, reference_features) (search/verifier.py:235-240).

    python tools/gen_golden_verifier_branches.py   ->  tests/golden/verifier_branches.npz
"""
import contextlib
import io
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np
import torch

import gen_golden as G


def main():
    G._stub_torchvision()
    with contextlib.redirect_stdout(io.StringIO()):
        V = G._load("ref_verifier", "search/verifier.py")
    g = torch.Generator().manual_seed(11)
    out = {}
    stats = {"mu": np.zeros(4), "sigma": np.eye(4)}
    for k, im in {"b1": torch.randn(1, 3, 32, 32, generator=g).clamp(-1, 1),
                  "b3": torch.rand(3, 3, 32, 32, generator=g) * 2 - 0.7,
                  "b2_64": torch.randn(2, 3, 64, 64, generator=g)}.items():
        out[k + "_images"] = im
        out[k + "_oracle_stats"] = np.float64(V.OracleVerifier(dataset_stats=stats).score(im))
    sv = V.SelfSupervisedVerifier()
    for k, shape in {"p32": (1, 3, 32, 32), "p64": (1, 3, 64, 64)}.items():
        im = torch.randn(*shape, generator=g)
        ref = torch.randn(1, 3 * 64, generator=g)
        out[k + "_images"] = im
        out[k + "_ref"] = ref
        out[k + "_paired"] = np.float64(sv.score(im, reference_features=ref))
    G.save("verifier_branches", **out)


if __name__ == "__main__":
    main()
