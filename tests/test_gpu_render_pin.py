"""The hot path pinned end-to-end to the reference's own output: the README experiment
(README.md:69-79) -- the template-API sample (samples/mlp_learning_an_image.hip, the reference's
samples/mlp_learning_an_image.cu:101-317) learning the full-resolution albert image (stb_image decode,
tests/golden/albert_full.png) with data/config_hash.json, B = 2^18, default_rng_t{1337} batches,
Trainer seed 1337, 8-bit-weight bilinear targets -- renders after steps 0..100 and 0..1000, scored
like the reference's data/readme/{100,1000}.jpg (tests/golden/reference_renders.json).

Bands (sigma: seed-to-seed spread of this engine's render PSNR over 8 seed pairs, measured on an
MI355X by tools/render_spread.py, tests/golden/render_spread.json: 0.17 dB at 100 steps, 0.18 dB at
1000):
  * 100 steps: within 3 sigma of the CPU oracle's render of the same run (same seeds, same targets;
    tests/golden/oracle_render.json) -- the GPU arithmetic reproduces the oracle over 101 steps at
    full scale;
  * 100 and 1000 steps: no worse than the reference's render (>= reference - 3 sigma) and at most
    1 dB (100) / 1.5 dB (1000) better. The measured offset (+0.62 / +0.86 dB) is reproduced by the
    CPU oracle in both its ideal and reference-mimic (fp16-accumulation) modes, so it is not this
    engine's arithmetic.
"""
import json
import os
import subprocess

import pytest

import render_metrics as RM

pytestmark = pytest.mark.gpu
BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "neuralbtf-tiny-cuda-nn_amd", "bin",
                   "mlp_learning_an_image")


def _json(name):
    with open(os.path.join(RM.GOLD, name)) as f:
        return json.load(f)


def test_readme_experiment_renders_match_reference(tmp_path):
    assert os.path.exists(BIN), "build the sample first (make -C neuralbtf-tiny-cuda-nn_amd)"
    img = RM.load_albert_full()
    pgm = str(tmp_path / "albert.pgm")
    RM.write_pgm(pgm, img)
    env = {k: v for k, v in os.environ.items() if not k.startswith("TCNN_SAMPLE_")}
    out = subprocess.run([BIN, pgm, os.path.join(RM.GOLD, "config_hash.json"), "1001"], capture_output=True, text=True,
                         timeout=300, cwd=tmp_path, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    got = {s: RM.psnr_gray(RM.read_pnm(str(tmp_path / f"{s}.ppm")), img) for s in (100, 1000)}
    ref = _json("reference_renders.json")["psnr_gray"]
    spread = _json("render_spread.json")["stats"]
    oracle = _json("oracle_render.json")["ideal"]["psnr_gray_100"]
    s100, s1000 = spread["100"]["std"], spread["1000"]["std"]
    print(f"render PSNR: 100 steps {got[100]:.3f} dB (reference {ref['100']:.3f}, oracle {oracle:.3f}), "
          f"1000 steps {got[1000]:.3f} dB (reference {ref['1000']:.3f})")
    assert abs(got[100] - oracle) <= 3 * s100, (got[100], oracle, s100)
    assert ref["100"] - 3 * s100 <= got[100] <= ref["100"] + 1.0, (got[100], ref["100"])
    assert ref["1000"] - 3 * s1000 <= got[1000] <= ref["1000"] + 1.5, (got[1000], ref["1000"])
