// tiny-cuda-nn/common.h -- shared definitions of the C++ template API (reference
// include/tiny-cuda-nn/common.h:115-235, common_host.h:71-110) for the MI355X engine.
//
// The template API (config.h, trainer.h, network_with_input_encoding.h, gpu_matrix.h, gpu_memory.h,
// random.h, loss.h, optimizer.h, common_device.h) is header-only over the C-ABI of
// libtcnn_mi355x.so (include/tcnn_mi355x.h): a program written against the reference's tcnn:: names
// (create_from_config, Trainer::training_step, network->inference, GPUMatrix, GPUMemory,
// generate_random_uniform, default_rng_t, linear_kernel) compiles with hipcc and links the engine.
// Streams are hipStream_t (the reference's cudaStream_t); errors are std::runtime_error, as the
// reference's CHECK_THROW / CUDA_CHECK_THROW raise.
#pragma once

#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include <json.hpp>  // nlohmann::json (the reference includes it as <json/json.hpp>)

#include "../tcnn_mi355x.h"

namespace tcnn {

using json = nlohmann::json;

// common.h:115-116: parameters / activations of the networks are half precision
using network_precision_t = __half;

// common.h:235: batch sizes must be multiples of this
static constexpr uint32_t BATCH_SIZE_GRANULARITY = 256;

// The reference records the CUDA SM it was compiled for; this build targets gfx950 only.
static constexpr uint32_t MIN_GPU_ARCH = 950;

// common.h:157-167: data matrices are RowMajor == SoA, ColumnMajor == AoS
enum class MatrixLayout {
	RowMajor = 0,
	SoA = 0,
	ColumnMajor = 1,
	AoS = 1,
};
static constexpr MatrixLayout RM = MatrixLayout::RowMajor;
static constexpr MatrixLayout SoA = MatrixLayout::SoA;
static constexpr MatrixLayout CM = MatrixLayout::ColumnMajor;
static constexpr MatrixLayout AoS = MatrixLayout::AoS;

// common.h:176-180
enum class GradientMode {
	Ignore,
	Overwrite,
	Accumulate,
};

// cpp_api.h:40-47: base of every forward context (unique_ptr-owned, not copyable)
struct Context {
	Context() = default;
	virtual ~Context() {}
	Context(const Context&) = delete;
	Context& operator=(const Context&) = delete;
	Context(Context&&) = delete;
	Context& operator=(Context&&) = delete;
};

template <typename T>
constexpr T div_round_up(T val, T divisor) {
	return (val + divisor - 1) / divisor;
}
template <typename T>
constexpr T next_multiple(T val, T divisor) {
	return div_round_up(val, divisor) * divisor;
}
template <typename T>
constexpr T previous_multiple(T val, T divisor) {
	return (val / divisor) * divisor;
}

// common_host.h:71-110
#define CHECK_THROW(x)                                                                                              \
	do {                                                                                                            \
		if (!(x)) throw std::runtime_error(std::string(__FILE__ ":" + std::to_string(__LINE__) + " check failed: " #x)); \
	} while (0)

#define HIP_CHECK_THROW(x)                                                                                                  \
	do {                                                                                                                    \
		hipError_t _result = (x);                                                                                           \
		if (_result != hipSuccess)                                                                                          \
			throw std::runtime_error(std::string(__FILE__ ":" + std::to_string(__LINE__) + " " #x " failed: ") +           \
			                         hipGetErrorString(_result));                                                       \
	} while (0)

namespace detail {
inline void check_rc(int rc) {
	if (rc != 0) throw std::runtime_error(tcnn_last_error());
}
template <class P>
inline P* check_handle(P* p) {
	if (!p) throw std::runtime_error(tcnn_last_error());
	return p;
}
}  // namespace detail

// common_host.h: device helpers
inline int cuda_device() { return tcnn_cuda_device(); }
inline void set_cuda_device(int device) { detail::check_rc(tcnn_set_cuda_device(device)); }
inline int cuda_device_count() {
	int n = 0;
	HIP_CHECK_THROW(hipGetDeviceCount(&n));
	return n;
}
// cuda_compute_capability(): the gfx architecture number of `device` (950 for an MI355X)
inline uint32_t cuda_compute_capability(int device = -1) {
	if (device < 0) device = cuda_device();
	hipDeviceProp_t p;
	HIP_CHECK_THROW(hipGetDeviceProperties(&p, device));
	const char* s = p.gcnArchName;  // "gfx950:sramecc+:xnack-"
	uint32_t v = 0;
	if (s[0] == 'g' && s[1] == 'f' && s[2] == 'x')
		for (const char* c = s + 3; *c && *c != ':'; ++c) v = v * 10 + (uint32_t)(*c >= '0' && *c <= '9' ? *c - '0' : 0);
	return v;
}

// gpu_memory.h:751-754: temporary device memory of the engine's workspaces (free_gpu_memory_arena
// of one stream: gpu_memory.h in this directory)
inline void free_all_gpu_memory_arenas() { tcnn_free_temporary_memory(); }

// common.h:232: the loss scale of half-precision training
template <typename T>
constexpr float default_loss_scale() {
	return sizeof(T) == 2 ? 128.0f : 1.0f;
}

}  // namespace tcnn
