// mlp_learning_an_image.hip -- the reference's sample application (samples/mlp_learning_an_image.cu)
// on the MI355X engine, written against the tcnn:: C++ template API (include/tiny-cuda-nn/config.h,
// trainer.h, gpu_matrix.h, gpu_memory.h, random.h, common_device.h): the library calls are the
// reference's, line for line -- create_loss / create_optimizer / NetworkWithInputEncoding / Trainer,
// generate_random_uniform with default_rng_t{1337}, trainer->training_step, trainer->loss,
// network->inference, free_all_gpu_memory_arenas. The application's own GPU code uses the HIP
// runtime where the reference uses CUDA's (stream). CDNA GPUs have no texture-sampling hardware
// (HIP marks tex2D unavailable for gfx950), so the image lookup is an explicit bilinear fetch with
// the semantics of the reference's texture (normalized coordinates, clamp addressing, linear filter
// at texel centres, and the texture unit's 8-bit fractional weights).
//
// Image I/O: the reference reads JPEG/EXR through stb_image and writes JPEGs; this repository has no
// image codec, so the image is a binary PGM (the full-resolution albert.jpg as decoded by the
// reference's stb_image, tests/golden/albert_full.png, tools/make_albert_full.py; or the 768x1024
// tests/golden/albert_768x1024.pgm), converted to RGBA float with the 2.2 gamma linearisation of
// stbi_loadf (stbi_wrapper.cpp:37-44), and learned images are written as PPM (the reference: JPEG q100).
//
//   mlp_learning_an_image <image.pgm> [config.json] [n_training_steps] [final_image.ppm]
//
// Test hooks (not in the reference): TCNN_SAMPLE_SEED replaces the batch RNG's seed 1337 and
// TCNN_SAMPLE_TRAINER_SEED the Trainer's parameter seed 1337 (tests/test_gpu_render_pin.py measures
// the seed-to-seed spread of the render PSNR with them); TCNN_SAMPLE_TEX_ROUND = rint (default) |
// trunc | exact selects how the bilinear fraction is held (the texture unit's 8 fractional bits,
// rounded or truncated, or fp32) and TCNN_SAMPLE_LOG2_BATCH replaces the batch size 2^18
// (tools/render_sweep.py varies them to look for the reference run's pipeline).
#include <tiny-cuda-nn/common_device.h>

#include <tiny-cuda-nn/config.h>

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

using namespace tcnn;
using precision_t = network_precision_t;

// stbi_loadf of an 8-bit grayscale image: RGBA float, (v / 255)^2.2 in RGB, alpha 1
GPUMemory<float> load_image(const std::string& filename, int& width, int& height) {
	std::ifstream f{filename, std::ios::binary};
	std::string magic;
	int maxval = 0;
	f >> magic >> width >> height >> maxval;
	f.get();
	if (!f || magic != "P5" || maxval != 255) throw std::runtime_error{"load_image: " + filename + " is not an 8-bit binary PGM"};
	std::vector<unsigned char> pix((size_t)width * height);
	f.read((char*)pix.data(), (std::streamsize)pix.size());
	if (!f) throw std::runtime_error{"load_image: " + filename + " is truncated"};
	std::vector<float> out((size_t)width * height * 4);
	for (size_t i = 0; i < pix.size(); ++i) {
		const float v = std::pow(pix[i] / 255.0f, 2.2f);
		out[4 * i + 0] = out[4 * i + 1] = out[4 * i + 2] = v;
		out[4 * i + 3] = 1.0f;
	}
	GPUMemory<float> result(out.size());
	result.copy_from_host(out.data());
	return result;
}

template <typename T>
__global__ void to_ldr(const uint64_t num_elements, const uint32_t n_channels, const uint32_t stride, const T* __restrict__ in,
                       uint8_t* __restrict__ out) {
	const uint64_t i = threadIdx.x + blockIdx.x * blockDim.x;
	if (i >= num_elements) return;
	const uint64_t pixel = i / n_channels;
	const uint32_t channel = i - pixel * n_channels;
	out[i] = (uint8_t)(powf(fmaxf(fminf(in[pixel * stride + channel], 1.0f), 0.0f), 1.0f / 2.2f) * 255.0f + 0.5f);
}

template <typename T>
void save_image(const T* image, int width, int height, int n_channels, int channel_stride, const std::string& filename) {
	GPUMemory<uint8_t> image_ldr(width * height * n_channels);
	linear_kernel(to_ldr<T>, 0, nullptr, (uint64_t)width * height * n_channels, (uint32_t)n_channels, (uint32_t)channel_stride, image,
	              image_ldr.data());
	std::vector<uint8_t> host(width * height * n_channels);
	HIP_CHECK_THROW(hipMemcpy(host.data(), image_ldr.data(), image_ldr.size(), hipMemcpyDeviceToHost));
	std::ofstream f{filename, std::ios::binary};
	f << "P6\n" << width << " " << height << "\n255\n";
	f.write((const char*)host.data(), (std::streamsize)host.size());
}

// the sample's image "texture": RGBA float, width x height, row-major
struct ImageTexture {
	const float4* data;
	int width, height;
	int round_mode;  // 0: rint to 1/256 (default), 1: truncate to 1/256, 2: fp32 fraction (test hook)
};

__device__ inline float tex_fraction(float f, int mode) {
	if (mode == 1) return floorf(f * 256.0f) * (1.0f / 256.0f);
	if (mode == 2) return f;
	return rintf(f * 256.0f) * (1.0f / 256.0f);
}

// tex2D<float4>(texture, u, v) with cudaFilterModeLinear, normalizedCoords, cudaAddressModeClamp:
// x_B = u * width - 0.5, i = floor(x_B), alpha = frac(x_B), tex = (1-a)(1-b) T[i,j] + a(1-b) T[i+1,j]
// + (1-a) b T[i,j+1] + a b T[i+1,j+1], alpha and beta held by the texture unit in 9-bit fixed point
// with 8 fractional bits (CUDA programming guide, "Texture Fetching", linear filtering); the rounding
// of the fraction to 1/256 is taken as round-to-nearest (the guide does not specify it)
__device__ inline float4 sample_bilinear(const ImageTexture& t, float u, float v) {
	const float x = u * t.width - 0.5f, y = v * t.height - 0.5f;
	const float fx = floorf(x), fy = floorf(y);
	const float ax = tex_fraction(x - fx, t.round_mode), ay = tex_fraction(y - fy, t.round_mode);
	const int x0 = min(max((int)fx, 0), t.width - 1), x1 = min(max((int)fx + 1, 0), t.width - 1);
	const int y0 = min(max((int)fy, 0), t.height - 1), y1 = min(max((int)fy + 1, 0), t.height - 1);
	const float4 a = t.data[y0 * t.width + x0], b = t.data[y0 * t.width + x1];
	const float4 c = t.data[y1 * t.width + x0], d = t.data[y1 * t.width + x1];
	const float w00 = (1.0f - ax) * (1.0f - ay), w10 = ax * (1.0f - ay), w01 = (1.0f - ax) * ay, w11 = ax * ay;
	return make_float4(w00 * a.x + w10 * b.x + w01 * c.x + w11 * d.x, w00 * a.y + w10 * b.y + w01 * c.y + w11 * d.y,
	                   w00 * a.z + w10 * b.z + w01 * c.z + w11 * d.z, w00 * a.w + w10 * b.w + w01 * c.w + w11 * d.w);
}

template <uint32_t stride>
__global__ void eval_image(uint32_t n_elements, ImageTexture texture, float* __restrict__ xs_and_ys, float* __restrict__ result) {
	uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n_elements) return;
	uint32_t output_idx = i * stride;
	uint32_t input_idx = i * 2;
	float4 val = sample_bilinear(texture, xs_and_ys[input_idx], xs_and_ys[input_idx + 1]);
	result[output_idx + 0] = val.x;
	result[output_idx + 1] = val.y;
	result[output_idx + 2] = val.z;
	for (uint32_t c = 3; c < stride; ++c) result[output_idx + c] = 1;
}

int main(int argc, char* argv[]) {
	try {
		uint32_t compute_capability = cuda_compute_capability();
		if (compute_capability < MIN_GPU_ARCH) {
			std::cerr << "Warning: Insufficient compute capability " << compute_capability << " detected. "
			          << "This program was compiled for >=" << MIN_GPU_ARCH << " and may thus behave unexpectedly." << std::endl;
		}

		if (argc < 2) {
			std::cout << "USAGE: " << argv[0] << " path-to-image.pgm [path-to-optional-config.json] [n_steps] [final.ppm]" << std::endl;
			std::cout << "Sample images: tests/golden/albert_768x1024.pgm, or albert_full.png converted to PGM." << std::endl;
			return 0;
		}

		json config = {
			{"loss", {{"otype", "RelativeL2"}}},
			{"optimizer", {{"otype", "Adam"}, {"learning_rate", 1e-2}, {"beta1", 0.9f}, {"beta2", 0.99f}, {"l2_reg", 0.0f}}},
			{"encoding", {{"otype", "OneBlob"}, {"n_bins", 32}}},
			{"network",
			 {{"otype", "FullyFusedMLP"}, {"n_neurons", 64}, {"n_hidden_layers", 4}, {"activation", "ReLU"}, {"output_activation", "None"}}},
		};

		if (argc >= 3) {
			std::cout << "Loading custom json config '" << argv[2] << "'." << std::endl;
			std::ifstream f{argv[2]};
			config = json::parse(std::string{std::istreambuf_iterator<char>{f}, std::istreambuf_iterator<char>{}});
		}

		// First step: load an image that we'd like to learn
		int width, height;
		GPUMemory<float> image = load_image(argv[1], width, height);

		// Second step: the image as a bilinear "texture", used to generate training data on the fly
		const char* round_env = std::getenv("TCNN_SAMPLE_TEX_ROUND");  // test hook, see the header
		const std::string round_mode = round_env ? round_env : "rint";
		if (round_mode != "rint" && round_mode != "trunc" && round_mode != "exact") throw std::runtime_error{"TCNN_SAMPLE_TEX_ROUND: rint | trunc | exact"};
		ImageTexture texture{(const float4*)image.data(), width, height, round_mode == "rint" ? 0 : round_mode == "trunc" ? 1 : 2};

		// Third step: sample a reference image to dump to disk
		int sampling_width = width;
		int sampling_height = height;

		uint32_t n_coords = sampling_width * sampling_height;
		uint32_t n_coords_padded = next_multiple(n_coords, BATCH_SIZE_GRANULARITY);

		GPUMemory<float> sampled_image(n_coords * 3);
		GPUMemory<float> xs_and_ys(n_coords_padded * 2);

		std::vector<float> host_xs_and_ys(n_coords * 2);
		for (int y = 0; y < sampling_height; ++y) {
			for (int x = 0; x < sampling_width; ++x) {
				int idx = (y * sampling_width + x) * 2;
				host_xs_and_ys[idx + 0] = (float)(x + 0.5) / (float)sampling_width;
				host_xs_and_ys[idx + 1] = (float)(y + 0.5) / (float)sampling_height;
			}
		}

		xs_and_ys.copy_from_host(host_xs_and_ys.data(), host_xs_and_ys.size());

		linear_kernel(eval_image<3>, 0, nullptr, n_coords, texture, xs_and_ys.data(), sampled_image.data());

		save_image(sampled_image.data(), sampling_width, sampling_height, 3, 3, "reference.ppm");

		// Fourth step: train the model by sampling the above image and optimizing an error metric
		const char* batch_env = std::getenv("TCNN_SAMPLE_LOG2_BATCH");  // test hook, see the header
		const uint32_t batch_size = 1u << (batch_env ? std::atoi(batch_env) : 18);
		const uint32_t n_training_steps = argc >= 4 ? atoi(argv[3]) : 10000000;
		const uint32_t n_input_dims = 2;   // 2-D image coordinate
		const uint32_t n_output_dims = 3;  // RGB color

		hipStream_t inference_stream;
		HIP_CHECK_THROW(hipStreamCreate(&inference_stream));
		hipStream_t training_stream = inference_stream;

		const char* seed_env = std::getenv("TCNN_SAMPLE_SEED");  // test hook, see the header
		default_rng_t rng{seed_env ? (uint64_t)std::strtoull(seed_env, nullptr, 10) : 1337u};

		// Auxiliary matrices for training
		GPUMatrix<float> training_target(n_output_dims, batch_size);
		GPUMatrix<float> training_batch(n_input_dims, batch_size);

		// Auxiliary matrices for evaluation
		GPUMatrix<float> prediction(n_output_dims, n_coords_padded);
		GPUMatrix<float> inference_batch(xs_and_ys.data(), n_input_dims, n_coords_padded);

		json encoding_opts = config.value("encoding", json::object());
		json loss_opts = config.value("loss", json::object());
		json optimizer_opts = config.value("optimizer", json::object());
		json network_opts = config.value("network", json::object());

		std::shared_ptr<Loss<precision_t>> loss{create_loss<precision_t>(loss_opts)};
		std::shared_ptr<Optimizer<precision_t>> optimizer{create_optimizer<precision_t>(optimizer_opts)};
		std::shared_ptr<NetworkWithInputEncoding<precision_t>> network =
		    std::make_shared<NetworkWithInputEncoding<precision_t>>(n_input_dims, n_output_dims, encoding_opts, network_opts);

		const char* tseed_env = std::getenv("TCNN_SAMPLE_TRAINER_SEED");  // test hook, see the header
		auto trainer = std::make_shared<Trainer<float, precision_t, precision_t>>(
		    network, optimizer, loss, tseed_env ? (uint32_t)std::strtoul(tseed_env, nullptr, 10) : 1337u);

		std::chrono::steady_clock::time_point begin = std::chrono::steady_clock::now();

		float tmp_loss = 0;
		uint32_t tmp_loss_counter = 0;

		std::cout << "Beginning optimization with " << n_training_steps << " training steps." << std::endl;

		uint32_t interval = 10;

		for (uint32_t i = 0; i < n_training_steps; ++i) {
			bool print_loss = i % interval == 0;
			bool visualize_learned_func = argc < 5 && i % interval == 0;

			// Compute reference values at random coordinates
			{
				generate_random_uniform<float>(training_stream, rng, batch_size * n_input_dims, training_batch.data());
				linear_kernel(eval_image<n_output_dims>, 0, training_stream, batch_size, texture, training_batch.data(), training_target.data());
			}

			// Training step
			{
				auto ctx = trainer->training_step(training_stream, training_batch, training_target);

				if (i % std::min(interval, (uint32_t)100) == 0) {
					tmp_loss += trainer->loss(training_stream, *ctx);
					++tmp_loss_counter;
				}
			}

			// Debug outputs
			{
				if (print_loss) {
					std::chrono::steady_clock::time_point end = std::chrono::steady_clock::now();
					std::cout << "Step#" << i << ": " << "loss=" << tmp_loss / (float)tmp_loss_counter
					          << " time=" << std::chrono::duration_cast<std::chrono::microseconds>(end - begin).count() << "[µs]" << std::endl;

					tmp_loss = 0;
					tmp_loss_counter = 0;
				}

				if (visualize_learned_func) {
					network->inference(inference_stream, inference_batch, prediction);
					auto filename = std::to_string(i) + ".ppm";
					std::cout << "Writing '" << filename << "'... ";
					save_image(prediction.data(), sampling_width, sampling_height, 3, n_output_dims, filename);
					std::cout << "done." << std::endl;
				}

				// Don't count visualizing as part of timing
				if (print_loss) begin = std::chrono::steady_clock::now();
			}

			if (print_loss && i > 0 && interval < 1000) interval *= 10;
		}

		// Dump final image if a name was specified
		if (argc >= 5) {
			network->inference(inference_stream, inference_batch, prediction);
			save_image(prediction.data(), sampling_width, sampling_height, 3, n_output_dims, argv[4]);
		}

		free_all_gpu_memory_arenas();
		HIP_CHECK_THROW(hipStreamDestroy(inference_stream));
	} catch (const std::exception& e) {
		std::cout << "Uncaught exception: " << e.what() << std::endl;
		return EXIT_FAILURE;
	}

	return EXIT_SUCCESS;
}
