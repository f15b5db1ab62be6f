"""The reference's C++ template API (create_from_config, Trainer::training_step / loss,
network->inference, GPUMatrix, GPUMemory, generate_random_uniform, default_rng_t) over the engine:
tests/cpp/template_api_consumer.cpp is built by the Makefile against include/tiny-cuda-nn/*.h and run
here on the GPU; a CPU test checks the headers declare the reference's interface."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd", "bin", "template_api_consumer")
INC = os.path.join(REPO, "include", "tiny-cuda-nn")


@pytest.mark.gpu
def test_template_api_consumer_runs():
    assert os.path.exists(BIN), "build it with make -C neuralbtf-tiny-cuda-nn_amd"
    r = subprocess.run([BIN, os.path.join(REPO, "tests", "golden", "config_hash.json")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "template api ok" in r.stdout, r.stdout


def test_template_headers_declare_reference_interface():
    want = {
        "config.h": ["struct TrainableModel", "create_from_config(uint32_t n_input_dims, uint32_t n_output_dims, json config)"],
        "trainer.h": ["class Trainer", "struct ForwardContext", "training_step(hipStream_t stream", "float loss(hipStream_t stream",
                      "void optimizer_step(hipStream_t stream, float loss_scale)", "params_full_precision()",
                      "set_params_full_precision(", "void update_hyperparams(const json& params)", "void initialize_params()",
                      "std::unique_ptr<ForwardContext> forward(hipStream_t stream, const float loss_scale",
                      "void backward(hipStream_t stream, const ForwardContext& ctx"],
        "network_with_input_encoding.h": ["class NetworkWithInputEncoding", "public DifferentiableObject<float, T, T>",
                                          "padded_output_width()", "size_t n_params()"],
        "object.h": ["class DifferentiableObject", "void inference(hipStream_t stream", "virtual uint32_t input_width()",
                     "virtual uint32_t output_width()", "virtual size_t n_params()"],
        "network.h": ["class Network : public DifferentiableObject<T, PARAMS_T, PARAMS_T>", "create_network(const json& network)",
                      "uint32_t width(uint32_t layer)", "num_forward_activations()"],
        "encoding.h": ["class Encoding", "create_encoding(uint32_t n_dims_to_encode"],
        "gpu_matrix.h": ["class GPUMatrixDynamic", "class GPUMatrix : public GPUMatrixDynamic<T>", "uint32_t m() const",
                         "uint32_t n() const", "transposed()"],
        "gpu_memory.h": ["class GPUMemory", "void copy_from_host(", "void copy_to_host(", "void resize(", "size_t get_bytes()",
                         "class GPUMemoryArena", "class Allocation", "allocate_workspace(hipStream_t stream, size_t n_bytes)",
                         "allocate_workspace_and_distribute(", "void free_gpu_memory_arena(hipStream_t stream)"],
        "multi_stream.h": ["struct SyncedMultiStream", "SyncedMultiStream(hipStream_t stream, size_t n_streams)",
                           "hipStream_t get(size_t idx)", "reserve_multi_stream(", "free_multi_streams("],
        "random.h": ["struct pcg32", "using default_rng_t = pcg32", "generate_random_uniform("],
        "common_device.h": ["linear_kernel(", "n_blocks_linear(", "N_THREADS_LINEAR"],
        "common.h": ["network_precision_t = __half", "BATCH_SIZE_GRANULARITY = 256", "enum class MatrixLayout",
                     "enum class GradientMode", "cuda_compute_capability(", "free_all_gpu_memory_arenas()", "MIN_GPU_ARCH"],
        "loss.h": ["class Loss", "create_loss("],
        "optimizer.h": ["class Optimizer", "create_optimizer("],
    }
    for f, syms in want.items():
        h = open(os.path.join(INC, f)).read()
        for s in syms:
            assert s in h, (f, s)
