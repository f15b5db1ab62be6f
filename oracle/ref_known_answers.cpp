// ref_known_answers.cpp -- TEST INFRASTRUCTURE. Includes the reference's own host-compilable headers
// (dependencies/pcg32/pcg32.h and include/tiny-cuda-nn/common.h, both compiled as they lie under
// /root/reference with g++, no stand-ins) and prints known answers as JSON. The output is committed
// as tests/golden/ref_known_answers.json and pins the oracle's RNG / seeding / Xavier / grid-table
// restatements (pcg32.h) and the engine's batch granularity, default loss scale and enum orders
// (common.h). Build + run: `make -C oracle ref` (writes only into oracle/_ref/).
//
// The strided loop below restates random.h:39-65 (CUDA-only, not compilable here) on top of the
// reference's pcg32; the level-resolution loop restates grid.h:688-719 with the reference's
// host-side expression (common_device.h:709-718 is CUDA-only).
#include <pcg32/pcg32.h>
#include <tiny-cuda-nn/common.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

using tcnn::pcg32;

static void print_arr(const char* name, const std::vector<float>& v, bool last = false) {
	std::printf("  \"%s\": [", name);
	for (size_t i = 0; i < v.size(); ++i) std::printf("%s%.9g", i ? ", " : "", v[i]);
	std::printf("]%s\n", last ? "" : ",");
}

static std::vector<float> strided_uniform(pcg32& rng, size_t n, float lo, float hi) {
	const size_t N_GEN = 4;
	size_t n_thr = (n + N_GEN - 1) / N_GEN;
	size_t n_threads = (n_thr + 127) / 128 * 128;
	std::vector<float> out(n);
	for (size_t i = 0; i < n_threads; ++i) {  // every launched thread writes (random.h:41-54)
		pcg32 r = rng;
		r.advance(i * N_GEN);
		for (size_t j = 0; j < N_GEN; ++j) {
			size_t idx = i + n_threads * j;
			if (idx >= n) break;
			out[idx] = std::fma(r.next_float(), hi - lo, lo);
		}
	}
	rng.advance(n);
	return out;
}

static std::vector<float> xavier(pcg32& rnd, uint32_t rows, uint32_t cols) {
	float scale = 1.0f;
	scale *= std::sqrt(6.0f / (float)(cols + rows));
	std::vector<float> v((size_t)rows * cols);
	for (size_t i = 0; i < v.size(); ++i) v[i] = (float)(rnd.next_float() * 2.0f * scale - scale);
	return v;
}

static std::vector<float> ends(const std::vector<float>& v, size_t k) {
	std::vector<float> r;
	for (size_t i = 0; i < k && i < v.size(); ++i) r.push_back(v[i]);
	for (size_t i = v.size() >= k ? v.size() - k : 0; i < v.size(); ++i) r.push_back(v[i]);
	return r;
}

int main() {
	std::printf("{\n");
	// common.h:126-170, 229-241: the constants and enum orders the engine's C-ABI and JSON parser mirror
	std::printf("  \"common_h\": {\"batch_size_granularity\": %u, \"n_threads_linear\": %u, \"default_loss_scale_float\": %.9g, "
	            "\"activation\": {\"ReLU\": %d, \"LeakyReLU\": %d, \"Exponential\": %d, \"Sine\": %d, \"Sigmoid\": %d, "
	            "\"Squareplus\": %d, \"Softplus\": %d, \"Tanh\": %d, \"None\": %d}, "
	            "\"grid_type\": {\"Hash\": %d, \"Dense\": %d, \"Tiled\": %d}, "
	            "\"hash_type\": {\"Prime\": %d, \"CoherentPrime\": %d, \"ReversedPrime\": %d, \"Rng\": %d}, "
	            "\"interpolation\": {\"Nearest\": %d, \"Linear\": %d, \"Smoothstep\": %d}},\n",
	            tcnn::BATCH_SIZE_GRANULARITY, tcnn::N_THREADS_LINEAR, tcnn::default_loss_scale<float>(),
	            (int)tcnn::Activation::ReLU, (int)tcnn::Activation::LeakyReLU, (int)tcnn::Activation::Exponential, (int)tcnn::Activation::Sine,
	            (int)tcnn::Activation::Sigmoid, (int)tcnn::Activation::Squareplus, (int)tcnn::Activation::Softplus, (int)tcnn::Activation::Tanh,
	            (int)tcnn::Activation::None, (int)tcnn::GridType::Hash, (int)tcnn::GridType::Dense, (int)tcnn::GridType::Tiled,
	            (int)tcnn::HashType::Prime, (int)tcnn::HashType::CoherentPrime, (int)tcnn::HashType::ReversedPrime, (int)tcnn::HashType::Rng,
	            (int)tcnn::InterpolationType::Nearest, (int)tcnn::InterpolationType::Linear, (int)tcnn::InterpolationType::Smoothstep);
	// trainer.h:52-55
	std::seed_seq seq{1337u};
	std::vector<uint32_t> seeds(2);
	seq.generate(seeds.begin(), seeds.end());
	std::printf("  \"seed_seq_1337\": [%u, %u],\n", seeds[0], seeds[1]);

	pcg32 r{1337};
	uint32_t u0 = r.next_uint();
	float f1 = r.next_float();
	std::printf("  \"pcg32_1337_next_uint\": %u,\n  \"pcg32_1337_next_float\": %.9g,\n", u0, f1);

	pcg32 adv{1337};
	adv.advance(1000003);
	std::printf("  \"pcg32_1337_advance_1000003_next_uint\": %u,\n", adv.next_uint());

	// Trainer::initialize_params for data/config_hash.json (W64, H2, grid L16 F2 log2T15 s1.5):
	// MLP Xavier on the host (fully_fused_mlp.cu:865-891), then grid uniform(-1e-4, 1e-4).
	pcg32 trng{seeds[0]};
	auto w0 = xavier(trng, 64, 32);
	auto w1 = xavier(trng, 64, 64);
	auto wo = xavier(trng, 16, 64);
	print_arr("xavier_w0_ends16", ends(w0, 16));
	print_arr("xavier_w1_ends16", ends(w1, 16));
	print_arr("xavier_wout_ends16", ends(wo, 16));
	auto grid = strided_uniform(trng, 708368, -1e-4f, 1e-4f);
	print_arr("grid_init_ends64", ends(grid, 64));
	double s = 0.0;
	for (float x : grid) s += x;
	std::printf("  \"grid_init_sum\": %.17g,\n", s);
	std::printf("  \"trainer_rng_after_init_next_uint\": %u,\n", trng.next_uint());

	// samples/mlp_learning_an_image.cu:222,258: default_rng_t rng{1337}; 2^18 x 2 batch floats
	pcg32 brng{1337};
	auto batch = strided_uniform(brng, (size_t)1 << 19, 0.0f, 1.0f);
	print_arr("batch_2p19_ends64", ends(batch, 64));
	std::printf("  \"batch_rng_after_next_uint\": %u,\n", brng.next_uint());

	// Level scales / resolutions (grid.h:694 host expression), config_hash (s=1.5) and s=2.0.
	for (int cfg = 0; cfg < 2; ++cfg) {
		float pls = cfg == 0 ? 1.5f : 2.0f;
		std::printf("  \"grid_levels_s%s\": [", cfg == 0 ? "1_5" : "2_0");
		for (uint32_t l = 0; l < 16; ++l) {
			float sc = exp2f(l * std::log2(pls)) * 16 - 1.0f;
			uint32_t res = (uint32_t)ceilf(sc) + 1;
			std::printf("%s[%.9g, %u]", l ? ", " : "", sc, res);
		}
		std::printf("]%s\n", cfg == 0 ? "," : "");
	}
	std::printf("}\n");
	return 0;
}
