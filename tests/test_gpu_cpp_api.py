"""Source compatibility of the reference's C++ runtime API ("keep the C++ tcnn::cpp
header"): tests/cpp/cpp_api_consumer.cpp is written against tcnn::cpp (reference cpp_api.h:50-117)
and built by the Makefile against include/tiny-cuda-nn/cpp_api.h + libtcnn_mi355x.so."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd", "bin", "cpp_api_consumer")


@pytest.mark.gpu
def test_cpp_api_consumer_runs():
    assert os.path.exists(BIN), "build it with make -C neuralbtf-tiny-cuda-nn_amd"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cpp_api ok: NetworkWithInputEncoding / GridEncoding" in r.stdout, r.stdout


def test_cpp_api_header_declares_reference_interface():
    h = open(os.path.join(REPO, "include", "tiny-cuda-nn", "cpp_api.h")).read()
    for sym in ["batch_size_granularity()", "cuda_device()", "set_cuda_device(", "free_temporary_memory()", "has_networks()",
                "default_loss_scale(", "preferred_precision()", "set_log_callback(", "struct Context", "class Module",
                "virtual void inference(", "virtual Context forward(", "virtual void backward(",
                "virtual void backward_backward_input(", "create_network_with_input_encoding(", "create_network(",
                "create_encoding("]:
        assert sym in h, sym
