// tiny-cuda-nn/random.h -- default_rng_t (= pcg32, reference common_device.h:331,
// dependencies/pcg32/pcg32.h), generate_random_uniform and generate_random_logistic (random.h:57-85)
// for the MI355X engine.
//
// pcg32: the PCG-XSH-RR 64/32 generator (O'Neill 2014) with the reference's conventions: default
// stream 1 (inc = 2 * initseq + 1), seeding by two steps around adding initstate, next_float() as the
// top 23 bits in [1, 2) minus 1, and a log-time jump-ahead. The engine's device kernel continues the
// same stream, so a batch generated here equals the reference sample's batch bit for bit.
#pragma once

#include "common.h"

namespace tcnn {

struct pcg32 {
	static constexpr uint64_t PCG32_DEFAULT_STATE = 0x853c49e6748fea9bULL;
	static constexpr uint64_t PCG32_DEFAULT_STREAM = 0xda3e39cb94b95bdbULL;
	static constexpr uint64_t PCG32_MULT = 0x5851f42d4c957f2dULL;

	uint64_t state = PCG32_DEFAULT_STATE, inc = PCG32_DEFAULT_STREAM;

	__host__ __device__ pcg32() {}
	__host__ __device__ explicit pcg32(uint64_t initstate, uint64_t initseq = 1u) { seed(initstate, initseq); }

	__host__ __device__ void seed(uint64_t initstate, uint64_t initseq = 1) {
		state = 0u;
		inc = (initseq << 1u) | 1u;
		next_uint();
		state += initstate;
		next_uint();
	}
	__host__ __device__ uint32_t next_uint() {
		const uint64_t old = state;
		state = old * PCG32_MULT + inc;
		const uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
		const uint32_t rot = (uint32_t)(old >> 59u);
		return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
	}
	__host__ __device__ uint32_t next_uint(uint32_t bound) {
		const uint32_t threshold = (~bound + 1u) % bound;
		for (;;) {
			const uint32_t r = next_uint();
			if (r >= threshold) return r % bound;
		}
	}
	__host__ __device__ float next_float() {
		union {
			uint32_t u;
			float f;
		} x;
		x.u = (next_uint() >> 9) | 0x3f800000u;
		return x.f - 1.0f;
	}
	// pcg32.h:139-158: multi-step advance in O(log delta)
	__host__ __device__ void advance(int64_t delta_) {
		uint64_t cur_mult = PCG32_MULT, cur_plus = inc, acc_mult = 1u, acc_plus = 0u;
		uint64_t delta = (uint64_t)delta_;  // a negative delta wraps around the 2^64 period
		while (delta > 0) {
			if (delta & 1) {
				acc_mult *= cur_mult;
				acc_plus = acc_plus * cur_mult + cur_plus;
			}
			cur_plus = (cur_mult + 1) * cur_plus;
			cur_mult *= cur_mult;
			delta /= 2;
		}
		state = acc_mult * state + acc_plus;
	}
	__host__ __device__ bool operator==(const pcg32& o) const { return state == o.state && inc == o.inc; }
	__host__ __device__ bool operator!=(const pcg32& o) const { return !(*this == o); }
};

using default_rng_t = pcg32;

// random.h:67-70: n_elements uniform values in [lower, upper) in the reference's strided order
// (4 per thread, thread i jumps 4 i steps), on the device; rng advances by n_elements.
inline void generate_random_uniform(hipStream_t stream, default_rng_t& rng, size_t n_elements, float* out, const float lower = 0.0f,
                                    const float upper = 1.0f) {
	detail::check_rc(tcnn_generate_random_uniform(stream, &rng.state, &rng.inc, (uint64_t)n_elements, out, lower, upper));
}
template <typename T, typename RNG>
void generate_random_uniform(hipStream_t stream, RNG& rng, size_t n_elements, T* out, const T lower = (T)0.0, const T upper = (T)1.0) {
	static_assert(std::is_same<T, float>::value, "generate_random_uniform: the engine generates float");
	generate_random_uniform(stream, (default_rng_t&)rng, n_elements, out, lower, upper);
}
template <typename T, typename RNG>
void generate_random_uniform(RNG& rng, size_t n_elements, T* out, const T lower = (T)0.0, const T upper = (T)1.0) {
	generate_random_uniform<T>(nullptr, rng, n_elements, out, lower, upper);
}

// random.h:77-85: logistic values (logit(u) * stddev * 0.551328895 + mean) over the same stream
inline void generate_random_logistic(hipStream_t stream, default_rng_t& rng, size_t n_elements, float* out, const float mean = 0.0f,
                                     const float stddev = 1.0f) {
	detail::check_rc(tcnn_generate_random_logistic(stream, &rng.state, &rng.inc, (uint64_t)n_elements, out, mean, stddev));
}
template <typename T, typename RNG>
void generate_random_logistic(hipStream_t stream, RNG& rng, size_t n_elements, T* out, const T mean = (T)0.0, const T stddev = (T)1.0) {
	static_assert(std::is_same<T, float>::value, "generate_random_logistic: the engine generates float");
	generate_random_logistic(stream, (default_rng_t&)rng, n_elements, out, mean, stddev);
}
template <typename T, typename RNG>
void generate_random_logistic(RNG& rng, size_t n_elements, T* out, const T mean = (T)0.0, const T stddev = (T)1.0) {
	generate_random_logistic<T>(nullptr, rng, n_elements, out, mean, stddev);
}

}  // namespace tcnn
