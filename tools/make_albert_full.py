"""Freeze the reference-held pin of the hot path (run in the build container, needs /root/reference).

1. Decodes data/images/albert.jpg (3250 x 4333, the sample's training image) with the reference's own
   stb_image (oracle/_ref/stbi_decode, built by `make -C oracle ref`) and stores the 8-bit pixels
   losslessly as tests/golden/albert_full.png -- the image the GPU box trains on.
2. Decodes the reference's renders data/readme/100.jpg and 1000.jpg (the sample's output after
   steps 0..100 and 0..1000 of data/config_hash.json, README.md:69-79) the same way and writes their
   PSNR against the training image to tests/golden/reference_renders.json.

Also recorded: how far PIL's libjpeg decode is from stb_image's, and the PSNR cost of the JPEG
quality-100 encode the reference's renders went through (save_stbi, stbi_wrapper.cpp:25-29) as
PIL's q100 round trip of the training image itself -- the part of a render's PSNR that is codec,
not training.

usage: python tools/make_albert_full.py
"""
import io
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
from PIL import Image

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import render_metrics as RM  # noqa: E402

REF = "/root/reference"
DEC = os.path.join(REPO, "oracle", "_ref", "stbi_decode")


def stbi(path, ch, tmp):
    out = os.path.join(tmp, os.path.basename(path) + (".pgm" if ch == 1 else ".ppm"))
    subprocess.check_call([DEC, path, out, str(ch)])
    return RM.read_pnm(out)


def main():
    if not os.path.exists(DEC):
        subprocess.check_call(["make", "-C", os.path.join(REPO, "oracle"), "ref"])
    with tempfile.TemporaryDirectory() as tmp:
        albert = stbi(os.path.join(REF, "data/images/albert.jpg"), 1, tmp)
        renders = {s: stbi(os.path.join(REF, f"data/readme/{s}.jpg"), 3, tmp) for s in (100, 1000)}
    assert albert.shape == (4333, 3250), albert.shape
    Image.fromarray(albert).save(RM.ALBERT_FULL, format="PNG", optimize=True)
    assert np.array_equal(RM.load_albert_full(), albert)

    pil = np.asarray(Image.open(os.path.join(REF, "data/images/albert.jpg")).convert("L"))
    d = pil.astype(np.int32) - albert
    buf = io.BytesIO()
    Image.fromarray(albert).save(buf, format="JPEG", quality=100)
    q100 = np.asarray(Image.open(io.BytesIO(buf.getvalue())))
    res = {
        "source": "data/readme/{100,1000}.jpg vs data/images/albert.jpg (README.md:69-79); sample "
                  "samples/mlp_learning_an_image.cu:252-288 renders after training steps 0..N (N + 1 steps)",
        "decoder": "reference stb_image.h (oracle/_ref/stbi_decode), renders decoded as RGB",
        "metric": "PSNR (dB) of the render's 8-bit luma (ITU-R 601 integer form, tests/render_metrics.py) "
                  "against the 8-bit gray training image, full 3250 x 4333",
        "psnr_gray": {str(s): RM.psnr_gray(r, albert) for s, r in renders.items()},
        "psnr_rgb": {str(s): RM.psnr(r, np.repeat(albert[..., None], 3, axis=2)) for s, r in renders.items()},
        "pil_vs_stbi_albert": {"max_abs": int(np.abs(d).max()), "frac_differing": float(np.mean(d != 0))},
        "jpeg_q100_roundtrip_psnr": RM.psnr(q100, albert),
        "image_shape_hw": list(albert.shape),
    }
    with open(RM.REFERENCE_RENDERS, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))
    print(RM.ALBERT_FULL, os.path.getsize(RM.ALBERT_FULL))


if __name__ == "__main__":
    main()
