// tiny-cuda-nn/common_device.h -- device-side helpers the reference's sample programs use
// (reference include/tiny-cuda-nn/common_device.h:42-60, 331): linear_kernel, n_blocks_linear,
// default_rng_t. The hash-grid / activation helpers of the reference's header are internal to the
// engine's kernels here (neuralbtf-tiny-cuda-nn_amd/csrc/grid_device.h) and not part of the API.
#pragma once

#include "common.h"
#include "gpu_matrix.h"
#include "gpu_memory.h"
#include "random.h"

namespace tcnn {

// common_device.h:42-60 (N_THREADS_LINEAR = 128)
static constexpr uint32_t N_THREADS_LINEAR = 128;
static constexpr uint32_t WARP_SIZE = 64;  // a CDNA wavefront

template <typename T>
constexpr uint32_t n_blocks_linear(T n_elements, uint32_t n_threads = N_THREADS_LINEAR) {
	return (uint32_t)div_round_up(n_elements, (T)n_threads);
}

template <typename K, typename T, typename... Types>
inline void linear_kernel(K kernel, uint32_t shmem_size, hipStream_t stream, T n_elements, Types... args) {
	if (n_elements <= 0) return;
	hipLaunchKernelGGL(kernel, dim3(n_blocks_linear(n_elements)), dim3(N_THREADS_LINEAR), shmem_size, stream, n_elements, args...);
	HIP_CHECK_THROW(hipGetLastError());
}

}  // namespace tcnn
