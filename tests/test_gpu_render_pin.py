"""The hot path pinned end-to-end to the reference's own output: the README experiment
(README.md:69-79) -- the template-API sample (samples/mlp_learning_an_image.hip, the reference's
samples/mlp_learning_an_image.cu:101-317) learning the full-resolution albert image (stb_image decode,
tests/golden/albert_full.png) with data/config_hash.json, default_rng_t{1337} batches, Trainer seed
1337, 8-bit-weight bilinear targets -- renders after steps 0..100 and 0..1000, compared with the
reference's data/readme/{100,1000}.jpg.

The reference's renders were made with batches of 2^16 points, not the 2^18 of today's sample
(r04: tools/render_crops.py + tools/render_compare.py ran the sample under one pipeline change at a
time and compared each render pixel by pixel with the reference's; only 2^16 reproduces the
reference's error pattern -- 42.5 dB render-to-render and residual correlation 0.971 at 100 steps,
against <= 35.2 dB / 0.84 for every other variant). At 2^16 the whole pipeline
-- pcg32 batches, initialisation, grid, fused MLP, loss, Adam -- runs the reference's run:

  * image PSNR within 3 sigma of the reference's render, both sides (sigma: this engine's seed
    spread at 2^16, tests/golden/render_spread_b16.json: 0.147 dB at 100 steps, 0.169 at 1000);
  * the render itself close to the reference's render (tests/golden/reference_render_crops.npz, a
    central 768 x 768 crop): PSNR and residual correlation above what any other seed pair of the
    same pipeline reaches (7 other pairs: <= 33.6 dB / 0.78 at 100 steps, <= 37.7 dB / 0.72 at 1000);
  * the CPU oracle's run at 2^16 (tools/make_oracle_render.py ideal 8 b16): the 100-step image PSNR
    within 3 sigma of the oracle's, and the render within 50 dB of the oracle's render crop
    (tests/golden/oracle_render_b16_crop.npz; measured 56.3 dB, residual correlation 0.999; the
    oracle itself sits at 42.5 dB / 0.972 from the reference's render, like this engine);
  * at the sample's 2^18 batch, the 100-step render within 3 sigma of the CPU oracle's render of the
    same run (tests/golden/oracle_render.json), as before.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import render_metrics as RM

pytestmark = pytest.mark.gpu
BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "neuralbtf-tiny-cuda-nn_amd", "bin",
                   "mlp_learning_an_image")


def _json(name):
    with open(os.path.join(RM.GOLD, name)) as f:
        return json.load(f)


def _run(tmp_path, img, log2_batch):
    pgm = str(tmp_path / "albert.pgm")
    if not os.path.exists(pgm):
        RM.write_pgm(pgm, img)
    env = {k: v for k, v in os.environ.items() if not k.startswith("TCNN_SAMPLE_")}
    env["TCNN_SAMPLE_LOG2_BATCH"] = str(log2_batch)
    out = subprocess.run([BIN, pgm, os.path.join(RM.GOLD, "config_hash.json"), "1001"], capture_output=True, text=True,
                         timeout=300, cwd=tmp_path, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    return {s: RM.read_pnm(str(tmp_path / f"{s}.ppm")) for s in ("100", "1000")}


def test_readme_experiment_reproduces_reference_renders(tmp_path):
    assert os.path.exists(BIN), "build the sample first (make -C neuralbtf-tiny-cuda-nn_amd)"
    img = RM.load_albert_full()
    renders = _run(tmp_path, img, 16)
    ref = _json("reference_renders.json")["psnr_gray"]
    spread = _json("render_spread_b16.json")["stats"]
    crops = RM.load_reference_crops()
    got = {s: RM.psnr_gray(renders[s], img) for s in renders}
    rr = {s: RM.render_vs_reference(renders[s], img, crops, s) for s in renders}
    print(f"batch 2^16: image PSNR 100 steps {got['100']:.3f} dB (reference {ref['100']:.3f}), 1000 steps "
          f"{got['1000']:.3f} dB (reference {ref['1000']:.3f}); render-to-render 100: {rr['100']}, 1000: {rr['1000']}")
    for s in ("100", "1000"):
        assert abs(got[s] - ref[s]) <= 3 * spread[s]["std"], (s, got[s], ref[s], spread[s]["std"])
    assert rr["100"]["psnr"] >= 40.0 and rr["100"]["residual_corr"] >= 0.93, rr["100"]
    assert rr["1000"]["psnr"] >= 38.5 and rr["1000"]["residual_corr"] >= 0.79, rr["1000"]
    # the same run on the CPU oracle
    oracle = _json("oracle_render.json")["ideal_b16"]["psnr_gray_100"]
    assert abs(got["100"] - oracle) <= 3 * spread["100"]["std"], (got["100"], oracle)
    z = np.load(os.path.join(RM.GOLD, "oracle_render_b16_crop.npz"))
    ours = RM.luma(renders["100"])[crops["rows"], crops["cols"]]
    vs_oracle = RM.psnr(ours, z["render_100"])
    print(f"render-to-render vs the oracle's run: {vs_oracle:.2f} dB")
    assert vs_oracle >= 50.0, vs_oracle


def test_sample_batch_render_matches_oracle(tmp_path):
    img = RM.load_albert_full()
    renders = _run(tmp_path, img, 18)
    got = RM.psnr_gray(renders["100"], img)
    oracle = _json("oracle_render.json")["ideal"]["psnr_gray_100"]
    s100 = _json("render_spread.json")["stats"]["100"]["std"]
    print(f"batch 2^18: 100 steps {got:.3f} dB (oracle {oracle:.3f})")
    assert abs(got - oracle) <= 3 * s100, (got, oracle, s100)
