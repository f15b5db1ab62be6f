"""The reference's sample application (samples/mlp_learning_an_image.cu) written against the tcnn::
template API (neuralbtf-tiny-cuda-nn_amd/samples/mlp_learning_an_image.hip): learns albert.jpg (the
committed 768x1024 PGM decode, tools/make_albert_fixture.py) with the reference configs as files,
prints the reference's progress lines, writes reference.ppm and the final image, and the loss falls."""
import os
import re
import subprocess

import pytest

from helpers import GOLD

pytestmark = pytest.mark.gpu
BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "neuralbtf-tiny-cuda-nn_amd", "bin",
                   "mlp_learning_an_image")
IMAGE = os.path.join(GOLD, "albert_768x1024.pgm")


@pytest.mark.parametrize("cfg", ["config_hash.json", "config_oneblob.json"])
def test_sample_trains_on_albert(cfg, tmp_path):
    assert os.path.exists(BIN), "build the sample first (make -C neuralbtf-tiny-cuda-nn_amd)"
    final = tmp_path / "final.ppm"
    out = subprocess.run([BIN, IMAGE, os.path.join(GOLD, cfg), "101", str(final)], capture_output=True, text=True, timeout=120,
                         cwd=tmp_path)
    assert out.returncode == 0, out.stdout + out.stderr
    losses = [float(m) for m in re.findall(r"Step#\d+: loss=([0-9.eE+-]+) time=\d+\[", out.stdout)]
    assert len(losses) == 3, out.stdout  # steps 0, 10, 100
    assert losses[-1] < 0.5 * losses[0], losses
    ref = (tmp_path / "reference.ppm").read_bytes()
    assert ref.startswith(b"P6\n768 1024\n255\n") and len(ref) == 16 + 768 * 1024 * 3
    img = final.read_bytes()
    assert img.startswith(b"P6\n768 1024\n255\n") and len(img) == len(ref)
    # the learned image resembles the reference: mean absolute 8-bit difference well below chance
    import numpy as np
    a = np.frombuffer(ref[16:], np.uint8).astype(np.float64)
    b = np.frombuffer(img[16:], np.uint8).astype(np.float64)
    assert np.mean(np.abs(a - b)) < 0.5 * np.mean(np.abs(a - a.mean())), (np.mean(np.abs(a - b)), np.mean(np.abs(a - a.mean())))
