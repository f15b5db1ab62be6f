"""The reference's sample driver (samples/mlp_learning_an_image.cu) rebuilt over the C-ABI
(neuralbtf-tiny-cuda-nn_amd/samples/mlp_learning_an_image.hip): runs the reference configs as
files, prints the reference's progress lines, and the loss falls."""
import os
import re
import subprocess

import pytest

from helpers import GOLD

pytestmark = pytest.mark.gpu
BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "neuralbtf-tiny-cuda-nn_amd", "bin",
                   "mlp_learning_an_image")


@pytest.mark.parametrize("cfg", ["config_hash.json", "config_oneblob.json"])
def test_sample_driver_trains(cfg):
    assert os.path.exists(BIN), "build the sample first (make -C neuralbtf-tiny-cuda-nn_amd)"
    out = subprocess.run([BIN, os.path.join(GOLD, cfg), "101"], capture_output=True, text=True, timeout=90)
    assert out.returncode == 0, out.stderr
    losses = [float(m) for m in re.findall(r"Step#\d+: loss=([0-9.eE+-]+) time=\d+\[", out.stdout)]
    assert len(losses) == 3, out.stdout  # steps 0, 10, 100
    assert losses[-1] < 0.5 * losses[0], losses
