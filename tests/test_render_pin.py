"""CPU side of the reference-held pin of the hot path: the README experiment (config_hash.json on the
full-resolution albert, B = 2^18, renders after 100 / 1000 steps; README.md:69-79,
samples/mlp_learning_an_image.cu:213-288).

  * tests/golden/reference_renders.json -- PSNR of the reference's own renders data/readme/{100,1000}.jpg
    against the training image, both decoded with the reference's stb_image (oracle/_ref/stbi_decode);
    re-derived here when /root/reference is present.
  * tests/golden/albert_full.png -- that decode of albert.jpg, the image the GPU test trains on.
  * tests/golden/oracle_render.json -- the CPU oracle running the same experiment for 101 steps
    (tools/make_oracle_render.py, ~10 min ideal, ~40 min mimic): per-step losses and the 100-step
    render PSNR, in the ideal mode (fp32 accumulation: what the GPU engine is checked against) and the
    reference-mimic mode (fp16 WMMA / CUTLASS accumulators and fp16 atomics). The
    first steps are re-run here and must reproduce the frozen losses exactly.

Finding (r04): the reference's renders were made with batches of 2^16 points, not
the sample's 2^18 (the only pipeline change that reproduces the reference's error pattern pixel by
pixel). At 2^18 the oracle sits +0.62 dB above the reference's render (the mimic mode moves it by only
+0.07 dB: not the reference's fp16 arithmetic); at 2^16 (key ideal_b16, 101 steps, ~4 min) the
oracle's render is within 0.03 dB of the reference's image PSNR and 42.5 dB from the reference's
render itself (residual correlation 0.972; other seed pairs of the same pipeline reach <= 33.6 dB /
0.78). The bands: the 2^16 oracle within 3 sigma of the reference's render (both sides, sigma of the
2^16 seed spread, tests/golden/render_spread_b16.json), its render within 40 dB / 0.93 of the
reference's; at 2^18 the mimic stays within 0.2 dB of the ideal.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import render_metrics as RM
from conftest import REPO
from oracle import oracle as O

REF = "/root/reference"
DEC = os.path.join(REPO, "oracle", "_ref", "stbi_decode")
HAVE_REF = os.path.isdir(REF) and os.path.exists(DEC)


def _json(name):
    with open(os.path.join(RM.GOLD, name)) as f:
        return json.load(f)


def sigma(step):
    return _json("render_spread.json")["stats"][str(step)]["std"]


@pytest.mark.skipif(not HAVE_REF, reason="needs /root/reference and oracle/_ref (make -C oracle ref)")
def test_reference_render_psnr_and_fixture_rederived(tmp_path):
    def dec(rel, ch):
        out = str(tmp_path / (os.path.basename(rel) + (".pgm" if ch == 1 else ".ppm")))
        subprocess.check_call([DEC, os.path.join(REF, rel), out, str(ch)], stdout=subprocess.DEVNULL)
        return RM.read_pnm(out)
    albert = dec("data/images/albert.jpg", 1)
    np.testing.assert_array_equal(albert, RM.load_albert_full())
    frozen = _json("reference_renders.json")
    for s in ("100", "1000"):
        assert RM.psnr_gray(dec(f"data/readme/{s}.jpg", 3), albert) == pytest.approx(frozen["psnr_gray"][s], abs=1e-9)


def test_reference_render_values():
    r = _json("reference_renders.json")
    assert r["psnr_gray"]["100"] == pytest.approx(28.316, abs=5e-3)
    assert r["psnr_gray"]["1000"] == pytest.approx(34.350, abs=5e-3)
    assert r["jpeg_q100_roundtrip_psnr"] > 55.0  # the renders' JPEG coding is noise far below their error


def _replay(mode, n_steps):
    cfg = json.load(open(os.path.join(RM.GOLD, "config_hash.json")))
    lin = RM.linearise(RM.load_albert_full())
    O.set_mimic(mode == "mimic")
    try:
        om = O.OracleModel(cfg, 2, 3, seed=1337)
        rng = O.pcg32(1337)
        B = 1 << (16 if mode.endswith("_b16") else 18)
        out = []
        for _ in range(n_steps):
            pos = O.generate_uniform(rng, 2 * B).reshape(B, 2)
            out.append(float(om.train_step(pos, RM.texture_targets(lin, pos), run_optimizer=True, n_threads=os.cpu_count())))
        return out
    finally:
        O.set_mimic(False)


@pytest.mark.parametrize("mode,n_steps", [("ideal", 2), ("mimic", 1), ("ideal_b16", 3)])
def test_oracle_render_trajectory_reproduces(mode, n_steps):
    frozen = _json("oracle_render.json")[mode]["losses"]
    assert len(frozen) == 101
    assert _replay(mode, n_steps) == frozen[:n_steps]


def test_oracle_render_psnr_against_reference():
    ref = _json("reference_renders.json")["psnr_gray"]["100"]
    o = _json("oracle_render.json")
    ideal, mimic = o["ideal"]["psnr_gray_100"], o["mimic"]["psnr_gray_100"]
    assert abs(mimic - ideal) <= 0.2, (mimic, ideal)
    # the reference's run (B = 2^16): image PSNR within 3 sigma both sides, and the render itself
    s16 = _json("render_spread_b16.json")["stats"]["100"]["std"]
    b16 = o["ideal_b16"]
    assert abs(b16["psnr_gray_100"] - ref) <= 3 * s16, (b16["psnr_gray_100"], ref, s16)
    rr = b16["vs_reference_render_100"]
    assert rr["psnr"] >= 40.0 and rr["residual_corr"] >= 0.93, rr
    # the losses fall like a trained model's (every mode)
    for m in ("ideal", "mimic", "ideal_b16"):
        l = o[m]["losses"]
        assert l[-1] < 0.01 * l[0], (m, l[0], l[-1])


def test_oracle_b16_crop_matches_reference_crop():
    """the frozen oracle crop against the frozen reference crop (same window, same luma)"""
    crops = RM.load_reference_crops()
    z = np.load(os.path.join(RM.GOLD, "oracle_render_b16_crop.npz"))
    assert RM.psnr(z["render_100"], crops["100"]) >= 40.0
