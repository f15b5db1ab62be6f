"""Freeze a central crop of the reference's own renders as a fixture (build container, needs
/root/reference and oracle/_ref/stbi_decode from `make -C oracle ref`).

data/readme/100.jpg and 1000.jpg are the reference sample's output (README.md:69-79) -- reference
data, decoded here with the reference's own stb_image, reduced to ITU-R 601 luma and cropped to the
768 x 768 window tools/render_crops.py uses -> tests/golden/reference_render_crops.npz. The GPU test
tests/test_gpu_render_pin.py compares this engine's renders of the same run with them pixel by pixel
(render-to-render PSNR and residual correlation), a far tighter pin than PSNR against the image.

usage: python tools/make_reference_render_crops.py
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import render_metrics as RM  # noqa: E402
from render_crops import CROP  # noqa: E402

DEC = os.path.join(REPO, "oracle", "_ref", "stbi_decode")


def main():
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for s in ("100", "1000"):
            o = os.path.join(tmp, s + ".ppm")
            subprocess.check_call([DEC, f"/root/reference/data/readme/{s}.jpg", o, "3"])
            out["render_" + s] = RM.luma(RM.read_pnm(o))[CROP]
    out["crop_rows"] = np.array([CROP[0].start, CROP[0].stop])
    out["crop_cols"] = np.array([CROP[1].start, CROP[1].stop])
    np.savez_compressed(os.path.join(RM.GOLD, "reference_render_crops.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
