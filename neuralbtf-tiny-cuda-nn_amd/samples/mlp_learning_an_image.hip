// mlp_learning_an_image.hip -- the reference's sample driver (samples/mlp_learning_an_image.cu) on the
// MI355X engine, through the C-ABI only (include/tcnn_mi355x.h): a 2D -> RGB image is learned by
// create_from_config() + training_step() at batch 2^18, printing the reference's progress lines
// ("Step#i: loss=... time=...[µs]", interval growing 10x up to 1000).
//
// Differences, on purpose: the image is procedural (no stb_image / albert.jpg in this repository),
// and training positions come from a counter-based hash on the device instead of pcg32 streams.
//
//   mlp_learning_an_image <config.json> [n_training_steps]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>

#include "tcnn_mi355x.h"

#define HIP_OK(x)                                                                        \
	do {                                                                                 \
		hipError_t e_ = (x);                                                             \
		if (e_ != hipSuccess) {                                                          \
			std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));          \
			return 1;                                                                    \
		}                                                                                \
	} while (0)
#define TCNN_OK(x)                                                                       \
	do {                                                                                 \
		if ((x) != 0) {                                                                  \
			std::fprintf(stderr, "%s failed: %s\n", #x, tcnn_last_error());              \
			return 1;                                                                    \
		}                                                                                \
	} while (0)

// procedural RGB "image" on [0,1)^2 (stands in for eval_image's bilinear texture fetch)
__device__ inline void image_rgb(float x, float y, float* rgb) {
	rgb[0] = 0.5f + 0.5f * sinf(9.0f * x) * cosf(7.0f * y);
	rgb[1] = 0.5f + 0.4f * sinf(23.0f * x * y + 1.0f);
	rgb[2] = 0.5f + 0.3f * cosf(31.0f * x) * sinf(17.0f * y) + 0.1f * (float)(((int)(x * 40.0f)) & 1);
}

__device__ inline float hash_uniform(uint32_t v) {
	v ^= v >> 16; v *= 0x7feb352dU; v ^= v >> 15; v *= 0x846ca68bU; v ^= v >> 16;
	return (float)(v >> 8) * (1.0f / 16777216.0f);
}

__global__ void make_batch(uint32_t n, uint32_t step, float* pos, float* target) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const float x = hash_uniform(2 * (i + step * n)), y = hash_uniform(2 * (i + step * n) + 1);
	pos[2 * i] = x;
	pos[2 * i + 1] = y;
	image_rgb(x, y, target + 3 * i);
}

int main(int argc, char** argv) {
	if (argc < 2) {
		std::printf("Usage: %s <config.json> [n_training_steps]\n", argv[0]);
		return 0;
	}
	std::ifstream f(argv[1]);
	if (!f) {
		std::fprintf(stderr, "cannot open %s\n", argv[1]);
		return 1;
	}
	std::stringstream ss;
	ss << f.rdbuf();
	const std::string config = ss.str();
	const uint32_t batch_size = 1u << 18;
	const uint32_t n_training_steps = argc >= 3 ? (uint32_t)std::atoi(argv[2]) : 1000u;
	const uint32_t n_input_dims = 2, n_output_dims = 3;

	hipStream_t stream;
	HIP_OK(hipStreamCreate(&stream));
	float *pos = nullptr, *target = nullptr;
	HIP_OK(hipMalloc(&pos, (size_t)batch_size * 2 * 4));
	HIP_OK(hipMalloc(&target, (size_t)batch_size * 3 * 4));

	tcnn_trainer* trainer = tcnn_trainer_create(n_input_dims, n_output_dims, config.c_str(), 1337);
	if (!trainer) {
		std::fprintf(stderr, "create_from_config failed: %s\n", tcnn_last_error());
		return 1;
	}
	std::printf("Beginning optimization with %u training steps (engine: %s).\n", n_training_steps, tcnn_trainer_engine(trainer));

	auto begin = std::chrono::steady_clock::now();
	float tmp_loss = 0.0f;
	uint32_t tmp_loss_counter = 0, interval = 10;
	for (uint32_t i = 0; i < n_training_steps; ++i) {
		const bool print_loss = i % interval == 0;
		hipLaunchKernelGGL(make_batch, dim3(batch_size / 256), dim3(256), 0, stream, batch_size, i, pos, target);
		TCNN_OK(tcnn_trainer_training_step(trainer, stream, batch_size, pos, target, 1));
		if (i % std::min(interval, 100u) == 0) {
			tmp_loss += tcnn_trainer_loss(trainer, stream);
			++tmp_loss_counter;
		}
		if (print_loss) {
			HIP_OK(hipStreamSynchronize(stream));
			const auto end = std::chrono::steady_clock::now();
			std::printf("Step#%u: loss=%g time=%lld[µs]\n", i, tmp_loss / (float)tmp_loss_counter,
			            (long long)std::chrono::duration_cast<std::chrono::microseconds>(end - begin).count());
			tmp_loss = 0.0f;
			tmp_loss_counter = 0;
			begin = std::chrono::steady_clock::now();
		}
		if (print_loss && i > 0 && interval < 1000) interval *= 10;
	}
	HIP_OK(hipStreamSynchronize(stream));
	tcnn_trainer_destroy(trainer);
	HIP_OK(hipFree(pos));
	HIP_OK(hipFree(target));
	HIP_OK(hipStreamDestroy(stream));
	return 0;
}
