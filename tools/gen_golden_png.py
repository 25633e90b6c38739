"""Golden geometry of the reference's own PNG grids (SampledImgs/*.png, written by torchvision
``save_image(x, path, nrow=8)`` at ``Diffusion/Train.py:839,843`` / ``TrainCondition.py:145,149``):
image size, PNG bit depth / colour type, and the largest value on the padding lines (2-pixel
separators of a 32-px grid). Pixel values themselves stay unpinned (no seeds or weights ship
with the reference). Writes tests/golden/png_grids.json; run in the build container only
(reads /root/reference as data).
"""
import json
import os
import struct
import sys

import numpy as np
from PIL import Image

REF = "/root/reference/SampledImgs"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "png_grids.json")


def main():
    res = {}
    for name in ("SampledGuidenceImgs.png", "NoisyGuidenceImgs.png", "SampledNoGuidenceImgs.png",
                 "NoisyNoGuidenceImgs.png"):
        path = os.path.join(REF, name)
        with open(path, "rb") as fh:
            head = fh.read(33)
        w, h = struct.unpack(">II", head[16:24])
        arr = np.asarray(Image.open(path).convert("RGB"))
        pad_rows = [r for r in range(h) if r % 34 in (0, 1)]
        pad_cols = [c for c in range(w) if c % 34 in (0, 1)]
        res[name] = {"width": w, "height": h, "bit_depth": head[24], "color_type": head[25],
                     "cols": (w - 2) // 34, "rows": (h - 2) // 34,
                     "padding_max": int(max(arr[pad_rows].max(), arr[:, pad_cols].max())),
                     "interior_max": int(arr.max())}
    with open(OUT, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    sys.exit(main())
