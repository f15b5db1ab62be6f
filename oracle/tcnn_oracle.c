/*
 * tcnn_oracle.c -- CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY: the parity
 * checker and the CPU baseline; never linked into the product. See tcnn_oracle.h for the contract.
 *
 * Compiled with -ffp-contract=off: every fused multiply-add below is an explicit fmaf() placed
 * where nvcc (default --fmad=true, no --use_fast_math: reference CMakeLists.txt:225,
 * bindings/torch/setup.py:110) contracts the reference's device expressions.
 */
#include "tcnn_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------------ */
/* fp16                                                                                        */
/* ------------------------------------------------------------------------------------------ */

uint16_t orc_f2h(float f) {
	uint32_t x;
	memcpy(&x, &f, 4);
	uint32_t sign = (x >> 16) & 0x8000u;
	uint32_t ax = x & 0x7fffffffu;
	if (ax >= 0x7f800000u) { /* inf / nan */
		return (uint16_t)(sign | 0x7c00u | (ax > 0x7f800000u ? 0x200u | ((ax >> 13) & 0x3ffu) : 0u));
	}
	if (ax >= 0x477ff000u) { /* rounds to >= 65520 -> inf */
		return (uint16_t)(sign | 0x7c00u);
	}
	if (ax < 0x38800000u) { /* result is subnormal (or zero) in fp16: value < 2^-14 */
		if (ax < 0x33000000u) { /* < 2^-25: rounds to zero (2^-25 exactly is a tie -> even 0) */
			return (uint16_t)sign;
		}
		uint32_t e = ax >> 23;                 /* biased exponent, 102..112 */
		uint32_t m = (ax & 0x7fffffu) | 0x800000u;
		uint32_t shift = 126 - e;              /* value = m * 2^(e-150); half ulp unit 2^-24 */
		uint32_t q = m >> shift;
		uint32_t rem = m & ((1u << shift) - 1u);
		uint32_t halfway = 1u << (shift - 1);
		if (rem > halfway || (rem == halfway && (q & 1u))) q++;
		return (uint16_t)(sign | q);
	}
	/* normal */
	uint32_t e = (ax >> 23) - 112;           /* rebias 127 -> 15 */
	uint32_t m = ax & 0x7fffffu;
	uint32_t q = (e << 10) | (m >> 13);
	uint32_t rem = m & 0x1fffu;
	if (rem > 0x1000u || (rem == 0x1000u && (q & 1u))) q++; /* carry into exponent is correct */
	return (uint16_t)(sign | q);
}

float orc_h2f(uint16_t h) {
	uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
	uint32_t e = (h >> 10) & 0x1fu;
	uint32_t m = h & 0x3ffu;
	uint32_t x;
	if (e == 0) {
		if (m == 0) {
			x = sign;
		} else { /* subnormal: normalise */
			int sh = 0;
			while (!(m & 0x400u)) { m <<= 1; ++sh; }
			m &= 0x3ffu;
			x = sign | ((uint32_t)(113 - sh) << 23) | (m << 13);
		}
	} else if (e == 31) {
		x = sign | 0x7f800000u | (m << 13);
	} else {
		x = sign | ((e + 112) << 23) | (m << 13);
	}
	float f;
	memcpy(&f, &x, 4);
	return f;
}

void orc_f2h_array(const float* in, uint16_t* out, size_t n) {
	for (size_t i = 0; i < n; ++i) out[i] = orc_f2h(in[i]);
}
void orc_h2f_array(const uint16_t* in, float* out, size_t n) {
	for (size_t i = 0; i < n; ++i) out[i] = orc_h2f(in[i]);
}

/* Round a double to fp16 (RNE). Used for the fp16 FMA emulation: a*b is exact in double and the
 * sum with c is exact whenever the exponent gap is below ~30 bits (always the case for the
 * grid's |w| <= 1 interpolation); the single rounding then equals __hfma/__hfma2. */
static uint16_t d2h(double d) {
	/* Convert via float only when that is exact; otherwise round directly. */
	float f = (float)d;
	if ((double)f == d) return orc_f2h(f);
	/* d is not representable in fp32: decide rounding on the double. Find the two fp16
	 * neighbours via the fp32-rounded value, then compare distances exactly in double. */
	uint16_t h = orc_f2h(f);
	double hv = (double)orc_h2f(h);
	if (hv == d) return h;
	/* neighbour in the direction of d */
	uint16_t n;
	int pos = d > hv;
	int neg_sign = (h & 0x8000u) != 0;
	if (h == 0x0000u || h == 0x8000u) {
		n = (uint16_t)(pos ? 0x0001u : 0x8001u);
	} else if (pos != neg_sign) {
		n = (uint16_t)(h + 1);
	} else {
		n = (uint16_t)(h - 1);
	}
	double nv = (double)orc_h2f(n);
	double dh = fabs(d - hv), dn = fabs(d - nv);
	if (dn < dh) return n;
	if (dn > dh) return h;
	return (n & 1u) ? h : n; /* tie: even mantissa */
}

uint16_t orc_hfma(uint16_t a, uint16_t b, uint16_t c) {
	return d2h((double)orc_h2f(a) * (double)orc_h2f(b) + (double)orc_h2f(c));
}

/* ------------------------------------------------------------------------------------------ */
/* PCG32 -- dependencies/pcg32/pcg32.h:40-200                                                  */
/* ------------------------------------------------------------------------------------------ */
#define PCG32_MULT 0x5851f42d4c957f2dULL

uint32_t orc_pcg32_next_uint(orc_pcg32* r) { /* pcg32.h:62-69 */
	uint64_t old = r->state;
	r->state = old * PCG32_MULT + r->inc;
	uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
	uint32_t rot = (uint32_t)(old >> 59u);
	return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
}

void orc_pcg32_seed(orc_pcg32* r, uint64_t initstate, uint64_t initseq) { /* pcg32.h:53-59 */
	r->state = 0u;
	r->inc = (initseq << 1u) | 1u;
	orc_pcg32_next_uint(r);
	r->state += initstate;
	orc_pcg32_next_uint(r);
}

float orc_pcg32_next_float(orc_pcg32* r) { /* pcg32.h:100-110 */
	uint32_t u = (orc_pcg32_next_uint(r) >> 9) | 0x3f800000u;
	float f;
	memcpy(&f, &u, 4);
	return f - 1.0f;
}

void orc_pcg32_advance(orc_pcg32* r, int64_t delta_) { /* pcg32.h:139-158 */
	uint64_t cur_mult = PCG32_MULT, cur_plus = r->inc, acc_mult = 1u, acc_plus = 0u;
	uint64_t delta = (uint64_t)delta_;
	while (delta > 0) {
		if (delta & 1) {
			acc_mult *= cur_mult;
			acc_plus = acc_plus * cur_mult + cur_plus;
		}
		cur_plus = (cur_mult + 1) * cur_plus;
		cur_mult *= cur_mult;
		delta /= 2;
	}
	r->state = acc_mult * r->state + acc_plus;
}

void orc_seed_seq(const uint32_t* v, size_t s, uint32_t* b, size_t n) {
	if (n == 0) return;
	for (size_t i = 0; i < n; ++i) b[i] = 0x8b8b8b8bu;
	size_t t = (n >= 623) ? 11 : (n >= 68) ? 7 : (n >= 39) ? 5 : (n >= 7) ? 3 : (n - 1) / 2;
	size_t p = (n - t) / 2, q = p + t;
	size_t m = (s + 1 > n) ? s + 1 : n;
	for (size_t k = 0; k < m; ++k) {
		uint32_t x = b[k % n] ^ b[(k + p) % n] ^ b[(k + n - 1) % n];
		uint32_t r1 = 1664525u * (x ^ (x >> 27));
		uint32_t r2;
		if (k == 0) r2 = r1 + (uint32_t)s;
		else if (k <= s) r2 = r1 + (uint32_t)(k % n) + v[k - 1];
		else r2 = r1 + (uint32_t)(k % n);
		b[(k + p) % n] += r1;
		b[(k + q) % n] += r2;
		b[k % n] = r2;
	}
	for (size_t k = m; k < m + n; ++k) {
		uint32_t x = b[k % n] + b[(k + p) % n] + b[(k + n - 1) % n];
		uint32_t r3 = 1566083941u * (x ^ (x >> 27));
		uint32_t r4 = r3 - (uint32_t)(k % n);
		b[(k + p) % n] ^= r3;
		b[(k + q) % n] ^= r4;
		b[k % n] = r4;
	}
}

/* random.h:39-70. generate_random_kernel<T, RNG, 4>: thread i advances by 4i and writes
 * out[i + n_threads*j]; n_threads = blocks*128 with blocks = ceil(ceil(n/4)/128). The transform
 * `val * (upper - lower) + lower` is a device lambda -> nvcc contracts it to one fma. */
void orc_generate_uniform(orc_pcg32* r, size_t n, float* out, float lo, float hi) {
	const size_t n_gen = 4;
	size_t n_thr_needed = (n + n_gen - 1) / n_gen;
	size_t n_threads = ((n_thr_needed + 127) / 128) * 128;
	float range = hi - lo;
	/* every one of the n_threads launched threads writes (random.h:41-54): the threads past
	 * n_thr_needed fill out[i + n_threads * j] too, from rng positions 4i.. beyond n */
	for (size_t i = 0; i < n_threads; ++i) {
		orc_pcg32 rr = *r;
		orc_pcg32_advance(&rr, (int64_t)(i * n_gen));
		for (size_t j = 0; j < n_gen; ++j) {
			size_t idx = i + n_threads * j;
			if (idx >= n) break;
			out[idx] = fmaf(orc_pcg32_next_float(&rr), range, lo);
		}
	}
	orc_pcg32_advance(r, (int64_t)n);
}

/* gpu_matrix.h:284-299 (fan_in = cols, fan_out = rows, gpu_matrix.h:227-231). Host code: no
 * contraction. */
void orc_xavier_uniform(orc_pcg32* r, uint32_t rows, uint32_t cols, float* out, float scale) {
	scale *= sqrtf(6.0f / (float)(cols + rows));
	size_t n = (size_t)rows * cols;
	for (size_t i = 0; i < n; ++i) {
		float t = orc_pcg32_next_float(r) * 2.0f;
		t = t * scale;
		out[i] = t - scale;
	}
}

/* ------------------------------------------------------------------------------------------ */
/* Grid encoding                                                                                */
/* ------------------------------------------------------------------------------------------ */

static uint32_t powi_u32(uint32_t base, uint32_t exp) {
	uint32_t r = 1;
	for (uint32_t i = 0; i < exp; ++i) r *= base;
	return r;
}

/* GridEncodingTemplated constructor, grid.h:668-730; grid_scale/grid_resolution
 * common_device.h:709-718. log2 is std::log2(float) on the host (grid.h:694, 784). */
int orc_grid_init(orc_grid* g) {
	uint32_t D = g->n_pos_dims, F = g->n_features_per_level, L = g->n_levels;
	if (L > ORC_MAX_LEVELS || D < 1 || D > 7 || F == 0) return -1;
	float log2_scale = log2f(g->per_level_scale);
	uint32_t offset = 0;
	for (uint32_t l = 0; l < L; ++l) {
		float scale = exp2f((float)l * log2_scale) * (float)g->base_resolution - 1.0f;
		uint32_t res = (uint32_t)ceilf(scale) + 1;
		uint32_t max_params = 0xffffffffu / 2;
		uint32_t params = powf((float)res, (float)D) > (float)max_params ? max_params : powi_u32(res, D);
		params = (params + 7u) / 8u * 8u;
		if (g->grid_type == ORC_GRID_TILED) {
			uint32_t t = powi_u32(g->base_resolution, D);
			if (t < params) params = t;
		} else if (g->grid_type == ORC_GRID_HASH) {
			uint32_t t = 1u << g->log2_hashmap_size;
			if (t < params) params = t;
		}
		g->scales[l] = scale;
		g->res[l] = res;
		g->offsets[l] = offset;
		offset += params;
	}
	g->offsets[L] = offset;
	g->n_params = offset * F;
	return 0;
}

/* common_device.h:631-655 */
static const uint32_t PRIMES[7] = {1958374283u, 2654435761u, 805459861u, 3674653429u, 2097192037u, 1434869437u, 2165219737u};
static const uint32_t COHERENT_PRIMES[7] = {1u, 2654435761u, 805459861u, 3674653429u, 2097192037u, 1434869437u, 2165219737u};
static const uint32_t REVERSED_PRIMES[7] = {2165219737u, 1434869437u, 2097192037u, 3674653429u, 805459861u, 2654435761u, 1958374283u};

uint32_t orc_coherent_prime_hash(uint32_t d, const uint32_t* pos_grid) {
	uint32_t r = 0;
	for (uint32_t i = 0; i < d; ++i) r ^= pos_grid[i] * COHERENT_PRIMES[i];
	return r;
}

/* grid_index, common_device.h:690-707 */
uint32_t orc_grid_index(const orc_grid* g, uint32_t level, const uint32_t* pos_grid) {
	uint32_t size = g->offsets[level + 1] - g->offsets[level];
	uint32_t res = g->res[level];
	uint32_t stride = 1, index = 0;
	for (uint32_t dim = 0; dim < g->n_pos_dims && stride <= size; ++dim) {
		index += pos_grid[dim] * stride;
		stride *= res;
	}
	if (g->grid_type == ORC_GRID_HASH && size < stride) {
		const uint32_t* pr = g->hash_type == ORC_HASH_PRIME ? PRIMES
			: g->hash_type == ORC_HASH_REVERSED_PRIME ? REVERSED_PRIMES : COHERENT_PRIMES;
		uint32_t r = 0;
		for (uint32_t i = 0; i < g->n_pos_dims; ++i) r ^= pos_grid[i] * pr[i];
		index = r;
	}
	return index % size;
}

/* pos_fract, common_device.h:841-868 (identity or smoothstep interpolation) */
static void pos_fract(float x, float scale, int smooth, float* pos, uint32_t* grid) {
	float p = fmaf(scale, x, 0.5f);
	float t = floorf(p);
	*grid = (uint32_t)(int)t;
	p -= t;
	if (smooth) { /* smoothstep, common_device.h:801-803: v*v*(3-2v); nvcc contracts 3-2v */
		p = p * p * fmaf(-2.0f, p, 3.0f);
	}
	*pos = p;
}

/* kernel_grid, grid.h:48-212 (encoded_positions part; dy_dx not restated here) */
float orc_random_val(uint32_t seed, uint32_t idx) {
	orc_pcg32 r;
	orc_pcg32_seed(&r, seed, 1u);
	orc_pcg32_advance(&r, (int64_t)idx);
	return orc_pcg32_next_float(&r);
}

/* max_level in levels for point i: (max_level * num_grid_features) / F (grid.h:69-73) */
static float orc_max_level(const orc_grid* g, uint32_t i) {
	const float ml = g->max_level_gpu ? g->max_level_gpu[i] : g->max_level;
	return (ml * (float)(g->n_levels * g->n_features_per_level)) / (float)g->n_features_per_level;
}
/* grid.h:75 (forward, dy_dx) masks level >= max_level + 1e-3; grid.h:242, 382, 488 (backwards) use > */
static int orc_masked_fwd(const orc_grid* g, uint32_t l, uint32_t i) { return g->opts && (float)l >= orc_max_level(g, i) + 1e-3f; }
static int orc_masked_bwd(const orc_grid* g, uint32_t l, uint32_t i) { return g->opts && (float)l > orc_max_level(g, i) + 1e-3f; }

void orc_grid_fwd(const orc_grid* g, uint32_t B, const float* pos_in, const uint16_t* table, uint16_t* enc) {
	const uint32_t D = g->n_pos_dims, F = g->n_features_per_level, L = g->n_levels;
	for (uint32_t l = 0; l < L; ++l) {
		const uint16_t* grid = table + (size_t)g->offsets[l] * F;
		const float scale = g->scales[l];
		for (uint32_t i = 0; i < B; ++i) {
			float pos[8];
			uint32_t pg[8], local[8];
			for (uint32_t d = 0; d < D; ++d) pos_fract(pos_in[(size_t)i * D + d], scale, g->interpolation == ORC_INTERP_SMOOTHSTEP, &pos[d], &pg[d]);
			uint16_t result[8] = {0};
			if (orc_masked_fwd(g, l, i)) {
				/* masked level: 0 */
			} else if (g->interpolation == ORC_INTERP_NEAREST) {
				uint32_t idx = orc_grid_index(g, l, pg) * F;
				for (uint32_t f = 0; f < F; ++f) result[f] = grid[idx + f];
			} else {
				for (uint32_t c = 0; c < (1u << D); ++c) {
					float w = 1.0f;
					for (uint32_t d = 0; d < D; ++d) {
						if ((c & (1u << d)) == 0) { w *= 1.0f - pos[d]; local[d] = pg[d]; }
						else { w *= pos[d]; local[d] = pg[d] + 1; }
					}
					uint16_t wh = orc_f2h(w);
					uint32_t idx = orc_grid_index(g, l, local) * F;
					for (uint32_t f = 0; f < F; ++f) result[f] = orc_hfma(wh, grid[idx + f], result[f]);
				}
			}
			for (uint32_t f = 0; f < F; ++f) enc[(size_t)(l * F + f) * B + i] = result[f];
		}
	}
}

/* kernel_grid_backward, grid.h:214-320, ideal precision (fp32 sums of exact products). */
/* ADD: one update of grid parameter (level base + p): the gradient sum, or (stats mode) the sum of
 * |update| and the number of updates per parameter -- the per-element tolerance of the GPU tests */
/* Reference-mimic mode: the reference accumulates in fp16 -- WMMA fragments
 * with __half accumulators in the fused MLP kernels (fully_fused_mlp.cu:68,198: one fp16 rounding of
 * the running sum per 16-deep K step), CUTLASS GEMMs with half_t accumulators (cutlass_matmul.h:67-68,
 * mma 16x8x8: one rounding per 8-deep K step; split-K slices of min(4096, B) samples whose partials
 * are reduced in half, fully_fused_mlp.cu:775), and the grid gradient through fp16 atomics into the
 * __half gradient buffer (grid.h:252-255,655-666). With the mode on the oracle rounds at those points
 * (the atomics in point order); off (default) it is the "ideal" fp32-accumulating restatement the GPU
 * engine is checked against. Used to size the gap between this engine and the reference's binary
 * (tests/golden/oracle_render.json). */
static int g_mimic = 0;
void orc_set_mimic(int on) { g_mimic = on; }
/* Magnitude mode of the MLP weight gradient (tests only): orc_mlp_bwd accumulates sum_i |delta_i a_i|
 * per weight instead of sum_i delta_i a_i (the deltas themselves are propagated as usual). It sizes
 * the per-element tolerance of a weight gradient: a perturbation of every term by e ulps moves the sum
 * by at most e 2^-10 times this magnitude. */
static int g_abs_wgrad = 0;
void orc_set_abs_wgrad(int on) { g_abs_wgrad = on; }
#define WTERM(x) (g_abs_wgrad ? fabsf(x) : (x))
/* magnitude mode also propagates the deltas through |W| (abs-backprop with the same ReLU masks), so
 * that the magnitude of a delta or of dL/dinput bounds what a one-ulp change of any upstream fp16
 * delta can move it, cancellation included */
#define DTERM(w, d) (g_abs_wgrad ? fabsf(w) * fabsf(d) : (w) * (d))
#define DABS(x) (g_abs_wgrad ? fabsf(x) : (x))
static inline float hround(float x) { return orc_h2f(orc_f2h(x)); }
/* fp16 running sum update after k products (chunked), see g_mimic */
#define MIMIC_STEP(acc, part, k, chunk, K) \
	do { if (g_mimic && (((k) + 1) % (chunk) == 0 || (k) + 1 == (K))) { (acc) = hround((acc) + (part)); (part) = 0.0f; } } while (0)

#define ADD(p, v) do { const float v_ = (v); if (grad) { if (g_mimic) grad[base + (p)] = hround(grad[base + (p)] + hround(v_)); \
	else grad[base + (p)] += v_; } \
	if (abssum) { abssum[base + (p)] += fabsf(v_); count[base + (p)] += 1; } } while (0)
static void grid_bwd_impl(const orc_grid* g, uint32_t B, const float* pos_in, const uint16_t* dL_dy, float* grad, float* abssum,
                          uint32_t* count) {
	const uint32_t D = g->n_pos_dims, F = g->n_features_per_level, L = g->n_levels;
	for (uint32_t l = 0; l < L; ++l) {
		const size_t base = (size_t)g->offsets[l] * F;
		const float scale = g->scales[l];
		for (uint32_t i = 0; i < B; ++i) {
			float pos[8], dy[8];
			uint32_t pg[8], local[8];
			for (uint32_t d = 0; d < D; ++d) pos_fract(pos_in[(size_t)i * D + d], scale, g->interpolation == ORC_INTERP_SMOOTHSTEP, &pos[d], &pg[d]);
			for (uint32_t f = 0; f < F; ++f) dy[f] = orc_h2f(dL_dy[(size_t)(l * F + f) * B + i]);
			if (orc_masked_bwd(g, l, i)) continue;
			if (g->interpolation == ORC_INTERP_NEAREST) {
				uint32_t idx = orc_grid_index(g, l, pg) * F;
				for (uint32_t f = 0; f < F; ++f) ADD(idx + f, dy[f]);
				continue;
			}
			if (g->opts && g->stochastic) { /* grid.h:284-298 */
				const float sample = orc_random_val(1337u, i + l * B);
				for (uint32_t d = 0; d < D; ++d) local[d] = sample >= pos[d] ? pg[d] : pg[d] + 1;
				uint32_t idx = orc_grid_index(g, l, local) * F;
				for (uint32_t f = 0; f < F; ++f) ADD(idx + f, dy[f]);
				continue;
			}
			for (uint32_t c = 0; c < (1u << D); ++c) {
				float w = 1.0f;
				for (uint32_t d = 0; d < D; ++d) {
					if ((c & (1u << d)) == 0) { w *= 1.0f - pos[d]; local[d] = pg[d]; }
					else { w *= pos[d]; local[d] = pg[d] + 1; }
				}
				float wh = orc_h2f(orc_f2h(w));
				uint32_t idx = orc_grid_index(g, l, local) * F;
				for (uint32_t f = 0; f < F; ++f) ADD(idx + f, wh * dy[f]);
			}
		}
	}
}

#undef ADD

void orc_grid_bwd(const orc_grid* g, uint32_t B, const float* pos_in, const uint16_t* dL_dy, float* grad) {
	grid_bwd_impl(g, B, pos_in, dL_dy, grad, NULL, NULL);
}

void orc_grid_bwd_stats(const orc_grid* g, uint32_t B, const float* pos_in, const uint16_t* dL_dy, float* abssum, uint32_t* count) {
	grid_bwd_impl(g, B, pos_in, dL_dy, NULL, abssum, count);
}

/* kernel_grid dy_dx branch (grid.h:171-211) + kernel_grid_backward_input (grid.h:322-349):
 * dL/dx[i][d] = sum_k dL/dy[k][i] * dy_dx[k][i][d], k = l*F + f ascending. nvcc contracts
 * `grads += weight * diff * pos_derivative` to fmaf(weight*diff, pos_derivative, grads) and
 * `result += dL_dy * dy_dx` to fmaf(dL_dy, dy_dx, result); written out explicitly. */
void orc_grid_bwd_input(const orc_grid* g, uint32_t B, const float* pos_in, const uint16_t* table, const uint16_t* dL_dy,
                        float* dL_dx) {
	const uint32_t D = g->n_pos_dims, F = g->n_features_per_level, L = g->n_levels;
	for (uint32_t i = 0; i < B; ++i) {
		float res[8] = {0};
		for (uint32_t l = 0; l < L; ++l) {
			if (orc_masked_fwd(g, l, i)) continue; /* dy_dx = 0 */
			const float scale = g->scales[l];
			float pos[8], pd[8];
			uint32_t pg[8], local[8];
			for (uint32_t d = 0; d < D; ++d) {
				float p = fmaf(scale, pos_in[(size_t)i * D + d], 0.5f);
				float t = floorf(p);
				pg[d] = (uint32_t)(int)t;
				p -= t;
				if (g->interpolation == ORC_INTERP_SMOOTHSTEP) {
					pd[d] = 6.0f * p * (1.0f - p);
					p = p * p * fmaf(-2.0f, p, 3.0f);
				} else {
					pd[d] = 1.0f;
				}
				pos[d] = p;
			}
			float grads[8][4];
			memset(grads, 0, sizeof(grads));
			if (g->interpolation != ORC_INTERP_NEAREST) {
				for (uint32_t gd = 0; gd < D; ++gd) {
					for (uint32_t idx = 0; idx < (1u << (D - 1)); ++idx) {
						float w = scale;
						for (uint32_t nd = 0; nd < D - 1; ++nd) {
							const uint32_t dim = nd >= gd ? nd + 1 : nd;
							if ((idx & (1u << nd)) == 0) { w *= 1.0f - pos[dim]; local[dim] = pg[dim]; }
							else { w *= pos[dim]; local[dim] = pg[dim] + 1; }
						}
						local[gd] = pg[gd];
						const uint32_t il = (g->offsets[l] + orc_grid_index(g, l, local)) * F;
						local[gd] = pg[gd] + 1;
						const uint32_t ir = (g->offsets[l] + orc_grid_index(g, l, local)) * F;
						for (uint32_t f = 0; f < F; ++f) {
							const float diff = orc_h2f(table[ir + f]) - orc_h2f(table[il + f]);
							grads[f][gd] = fmaf(w * diff, pd[gd], grads[f][gd]);
						}
					}
				}
			}
			for (uint32_t f = 0; f < F; ++f) {
				const float dy = orc_h2f(dL_dy[(size_t)(l * F + f) * B + i]);
				for (uint32_t d = 0; d < D; ++d) res[d] = fmaf(dy, grads[f][d], res[d]);
			}
		}
		for (uint32_t d = 0; d < D; ++d) dL_dx[(size_t)i * D + d] = res[d];
	}
}


/* pos_fract with first and second derivative (common_device.h:801-829) */
static void orc_pos_fract2(uint32_t interp, float x, float scale, float* p, float* pd, float* pd2, uint32_t* pg) {
	float v = fmaf(scale, x, 0.5f);
	const float t = floorf(v);
	*pg = (uint32_t)(int)t;
	v -= t;
	if (interp == ORC_INTERP_SMOOTHSTEP) {
		/* nvcc contracts a - b*c into one fma (its default --fmad=true) */
		*pd2 = fmaf(-12.0f, v, 6.0f);
		*pd = 6.0f * v * (1.0f - v);
		*p = v * v * fmaf(-2.0f, v, 3.0f);
	} else {
		*pd2 = 0.0f;
		*pd = 1.0f;
		*p = v;
	}
}

void orc_grid_bwd_bwd(const orc_grid* g, uint32_t B, const float* pos_in, const uint16_t* table, const float* dL_ddLdx,
                      const uint16_t* dL_dy, float* grad, float* dL_ddLdy, float* dL_dx) {
	const uint32_t D = g->n_pos_dims, F = g->n_features_per_level, L = g->n_levels;
	const int linear_like = g->interpolation != ORC_INTERP_NEAREST;
	for (uint32_t i = 0; i < B; ++i) {
		const float* gx = dL_ddLdx + (size_t)i * D;
		float dx[8] = {0};
		for (uint32_t l = 0; l < L; ++l) {
			const float scale = g->scales[l];
			float p[8], pd[8], pd2[8], dy[8];
			uint32_t pg[8], local[8];
			for (uint32_t d = 0; d < D; ++d) orc_pos_fract2(g->interpolation, pos_in[(size_t)i * D + d], scale, &p[d], &pd[d], &pd2[d], &pg[d]);
			for (uint32_t f = 0; f < F; ++f) dy[f] = dL_dy ? orc_h2f(dL_dy[(size_t)(l * F + f) * B + i]) : 0.0f;
			const uint32_t base = g->offsets[l] * F;
			const int mfwd = orc_masked_fwd(g, l, i), mbwd = orc_masked_bwd(g, l, i);
#define ORC_IDX(loc) (base + orc_grid_index(g, l, (loc)) * F)
			/* (1) dL/dgrid: grid.h:433-454 -- per gradient dim, the 2^(D-1) edges along it */
			if (grad && dL_dy && linear_like && !mbwd) {
				for (uint32_t gd = 0; gd < D; ++gd) {
					const float grad_in = scale * gx[gd] * pd[gd];
					for (uint32_t idx = 0; idx < (1u << (D - 1)); ++idx) {
						float w = grad_in;
						for (uint32_t nd = 0; nd < D - 1; ++nd) {
							const uint32_t dim = nd >= gd ? nd + 1 : nd;
							if ((idx & (1u << nd)) == 0) { w *= 1.0f - p[dim]; local[dim] = pg[dim]; }
							else { w *= p[dim]; local[dim] = pg[dim] + 1; }
						}
						local[gd] = pg[gd];
						const uint32_t il = ORC_IDX(local);
						local[gd] = pg[gd] + 1;
						const uint32_t ir = ORC_IDX(local);
						for (uint32_t f = 0; f < F; ++f) {
							grad[il + f] += -w * dy[f];
							grad[ir + f] += w * dy[f];
						}
					}
				}
			}
			/* (2) dL/d(dL/dy) = dy_dx . dL/d(dL/dx): dy_dx as kernel_grid computes it (grid.h:171-211) */
			if (dL_ddLdy) {
				for (uint32_t f = 0; f < F; ++f) {
					float r = 0.0f;
					if (linear_like && !mfwd) {
						for (uint32_t gd = 0; gd < D; ++gd) {
							float dydx = 0.0f;
							for (uint32_t idx = 0; idx < (1u << (D - 1)); ++idx) {
								float w = scale;
								for (uint32_t nd = 0; nd < D - 1; ++nd) {
									const uint32_t dim = nd >= gd ? nd + 1 : nd;
									if ((idx & (1u << nd)) == 0) { w *= 1.0f - p[dim]; local[dim] = pg[dim]; }
									else { w *= p[dim]; local[dim] = pg[dim] + 1; }
								}
								local[gd] = pg[gd];
								const float vl = orc_h2f(table[ORC_IDX(local) + f]);
								local[gd] = pg[gd] + 1;
								const float vr = orc_h2f(table[ORC_IDX(local) + f]);
								dydx += w * (vr - vl) * pd[gd];
							}
							r += dydx * gx[gd];
						}
					}
					dL_ddLdy[(size_t)i * L * F + l * F + f] = r;
				}
			}
			/* (3) dL/dx through the Hessian of y (grid.h:542-598) */
			if (dL_dx && dL_dy && linear_like && !mbwd) {
				for (uint32_t gd = 0; gd < D; ++gd) {
					float out = 0.0f;
					for (uint32_t idx = 0; idx < (1u << (D - 1)); ++idx) {
						if (g->interpolation == ORC_INTERP_SMOOTHSTEP) { /* diagonal part */
							float w = scale * scale * gx[gd] * pd2[gd];
							for (uint32_t nd = 0; nd < D - 1; ++nd) {
								const uint32_t dim = nd >= gd ? nd + 1 : nd;
								if ((idx & (1u << nd)) == 0) { w *= 1.0f - p[dim]; local[dim] = pg[dim]; }
								else { w *= p[dim]; local[dim] = pg[dim] + 1; }
							}
							local[gd] = pg[gd];
							const uint32_t il = ORC_IDX(local);
							local[gd] = pg[gd] + 1;
							const uint32_t ir = ORC_IDX(local);
							for (uint32_t f = 0; f < F; ++f)
								out += (orc_h2f(table[ir + f]) - orc_h2f(table[il + f])) * dy[f] * w;
						}
						for (uint32_t oo = 0; oo < D - 1; ++oo) { /* mixed part, d/dx_gd of dy/dx_od */
							const uint32_t od = oo >= gd ? oo + 1 : oo;
							float w = scale * scale * gx[od] * pd[od] * pd[gd];
							for (uint32_t nd = 0; nd < D - 1; ++nd) {
								const uint32_t dim = nd >= od ? nd + 1 : nd;
								if ((idx & (1u << nd)) == 0) {
									w *= dim != gd ? 1.0f - p[dim] : -1.0f;
									local[dim] = pg[dim];
								} else {
									if (dim != gd) w *= p[dim];
									local[dim] = pg[dim] + 1;
								}
							}
							local[od] = pg[od];
							const uint32_t il = ORC_IDX(local);
							local[od] = pg[od] + 1;
							const uint32_t ir = ORC_IDX(local);
							for (uint32_t f = 0; f < F; ++f)
								out += (orc_h2f(table[ir + f]) - orc_h2f(table[il + f])) * dy[f] * w;
						}
					}
					dx[gd] += out;
				}
			}
#undef ORC_IDX
		}
		if (dL_dx)
			for (uint32_t d = 0; d < D; ++d) dL_dx[(size_t)i * D + d] = dx[d];
	}
}

/* ------------------------------------------------------------------------------------------ */
/* Fully fused MLP                                                                              */
/* ------------------------------------------------------------------------------------------ */

/* NH == 0 (CutlassMLP without hidden layers, cutlass_mlp.cu:64-67): one [OUTP][IN] matrix */
uint32_t orc_mlp_n_params(uint32_t W, uint32_t IN, uint32_t NH, uint32_t OUTP) {
	if (NH == 0) return OUTP * IN;
	return W * IN + (NH - 1) * W * W + OUTP * W;
}

/* Activations (common_device.h:102-160, warp_activation; fp32 math on the fp32 accumulator, rounded
 * to fp16 by the caller). The activation argument of the MLP functions carries the hidden activation
 * in bits 0-7 and the output activation in bits 8-15 (Activation enum order, common.h:126-136:
 * None, ReLU, LeakyReLU, Exponential, Sine, Sigmoid, Squareplus, Softplus, Tanh). */
#define ORC_K_ACT 10.0f
static inline float act_fwd(uint32_t act, float x) {
	switch (act & 0xffu) {
		case 1: return x > 0.0f ? x : 0.0f;
		case 2: return x * (x > 0.0f ? 1.0f : 0.01f);
		case 3: return expf(x);
		case 4: return sinf(x);
		case 5: return 1.0f / (1.0f + expf(-x));
		case 6: { const float y = x * ORC_K_ACT; return 0.5f * (y + sqrtf(y * y + 4.0f)) / ORC_K_ACT; }
		case 7: return logf(expf(x * ORC_K_ACT) + 1.0f) / ORC_K_ACT;
		case 8: return tanhf(x);
		default: return x;
	}
}
/* Transfer given the post-activation value y (warp_activation_backward, common_device.h:240-297):
 * g * (T)factor(y) in fp16 -- both operands fp16, the product rounded once (exact in fp32 first).
 * ReLU / None pass the fp16 value of g unchanged or 0. Sine has no post-activation backward. */
static inline float act_bwd(uint32_t act, float g, float y) {
	const float gh = orc_h2f(orc_f2h(g));
	float f;
	switch (act & 0xffu) {
		case 0: return gh;
		case 1: return y > 0.0f ? gh : 0.0f;
		case 2: f = y > 0.0f ? 1.0f : 0.01f; break;
		case 3: f = y; break;
		case 5: f = y * orc_h2f(orc_f2h(1.0f - y)); break;
		case 6: { const float t = y * ORC_K_ACT; f = t * t / (t * t + 1.0f); break; }
		case 7: f = 1.0f - expf(-y * ORC_K_ACT); break;
		case 8: f = 1.0f - y * y; break;
		default: return gh;
	}
	return orc_h2f(orc_f2h(gh * orc_h2f(orc_f2h(f))));
}

void orc_act_bwd_output(uint32_t act, size_t n, const uint16_t* out16, uint16_t* g16) {
	const uint32_t a = (act >> 8) & 0xffu;
	if (a == 0) return;
	for (size_t i = 0; i < n; ++i) g16[i] = orc_f2h(act_bwd(a, orc_h2f(g16[i]), orc_h2f(out16[i])));
}

typedef struct {
	uint32_t W, IN, NH, OUTP;
	float* wf; /* fp32 copy of fp16 weights */
	size_t off[64];
} mlp_view;

static void mlp_view_init(mlp_view* v, uint32_t W, uint32_t IN, uint32_t NH, uint32_t OUTP, const uint16_t* params) {
	v->W = W; v->IN = IN; v->NH = NH; v->OUTP = OUTP;
	size_t n = orc_mlp_n_params(W, IN, NH, OUTP);
	v->wf = (float*)malloc(n * sizeof(float));
	orc_h2f_array(params, v->wf, n);
	size_t o = 0;
	v->off[0] = 0;
	if (NH == 0) return;  /* the output matrix at 0 */
	o += (size_t)W * IN;
	for (uint32_t k = 1; k < NH; ++k) { v->off[k] = o; o += (size_t)W * W; }
	v->off[NH] = o;
}

static inline float in_at(const uint16_t* input, int soa, uint32_t IN, uint32_t B, uint32_t i, uint32_t k) {
	return orc_h2f(soa ? input[(size_t)k * B + i] : input[(size_t)i * IN + k]);
}

/* one sample forward; h: NH*W floats (fp16-rounded post-activations); out: OUTP fp16 */
static void mlp_fwd_sample(const mlp_view* v, uint32_t act, const float* x, float* h, uint16_t* out) {
	const uint32_t W = v->W, IN = v->IN, NH = v->NH, OUTP = v->OUTP;
	if (NH == 0) {  /* out = act_out(Wout x) */
		const float* Wo = v->wf;
		for (uint32_t o = 0; o < OUTP; ++o) {
			float acc = 0.0f, part = 0.0f;
			for (uint32_t k = 0; k < IN; ++k) { part += Wo[(size_t)o * IN + k] * x[k]; MIMIC_STEP(acc, part, k, 16, IN); }
			if (!g_mimic) acc = part;
			out[o] = orc_f2h(act_fwd(act >> 8, acc));
		}
		return;
	}
	const float* W0 = v->wf + v->off[0];
	for (uint32_t n = 0; n < W; ++n) {
		float acc = 0.0f, part = 0.0f;
		for (uint32_t k = 0; k < IN; ++k) { part += W0[(size_t)n * IN + k] * x[k]; MIMIC_STEP(acc, part, k, 16, IN); }
		if (!g_mimic) acc = part;
		h[n] = orc_h2f(orc_f2h(act_fwd(act, acc)));
	}
	for (uint32_t l = 1; l < NH; ++l) {
		const float* Wl = v->wf + v->off[l];
		const float* hp = h + (size_t)(l - 1) * W;
		float* hn = h + (size_t)l * W;
		for (uint32_t n = 0; n < W; ++n) {
			float acc = 0.0f, part = 0.0f;
			for (uint32_t k = 0; k < W; ++k) { part += Wl[(size_t)n * W + k] * hp[k]; MIMIC_STEP(acc, part, k, 16, W); }
			if (!g_mimic) acc = part;
			hn[n] = orc_h2f(orc_f2h(act_fwd(act, acc)));
		}
	}
	const float* Wo = v->wf + v->off[NH];
	const float* hl = h + (size_t)(NH - 1) * W;
	for (uint32_t o = 0; o < OUTP; ++o) {
		float acc = 0.0f, part = 0.0f;
		for (uint32_t k = 0; k < W; ++k) { part += Wo[(size_t)o * W + k] * hl[k]; MIMIC_STEP(acc, part, k, 16, W); }
		if (!g_mimic) acc = part;
		out[o] = orc_f2h(act_fwd(act >> 8, acc));  /* output activation (last_layer_forward) */
	}
}

void orc_mlp_fwd(uint32_t W, uint32_t IN, uint32_t NH, uint32_t OUTP, uint32_t act,
                 const uint16_t* params, uint32_t B, const uint16_t* input, int input_soa,
                 uint16_t* out, uint16_t* hidden, int n_threads) {
	mlp_view v;
	mlp_view_init(&v, W, IN, NH, OUTP, params);
#ifdef _OPENMP
	if (n_threads <= 0) n_threads = 1;
#pragma omp parallel num_threads(n_threads)
#endif
	{
		float* x = (float*)malloc(sizeof(float) * IN);
		float* h = (float*)malloc(sizeof(float) * NH * W);
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
		for (int64_t ii = 0; ii < (int64_t)B; ++ii) {
			uint32_t i = (uint32_t)ii;
			for (uint32_t k = 0; k < IN; ++k) x[k] = in_at(input, input_soa, IN, B, i, k);
			mlp_fwd_sample(&v, act, x, h, out + (size_t)i * OUTP);
			if (hidden) {
				for (uint32_t l = 0; l < NH; ++l)
					for (uint32_t n = 0; n < W; ++n) hidden[(size_t)l * W * B + (size_t)i * W + n] = orc_f2h(h[(size_t)l * W + n]);
			}
		}
		free(x); free(h);
	}
	free(v.wf);
}

/* backward of one sample: g fp16 dL/dout (OUTP), h hidden (NH*W). Accumulates wgrad (fp32),
 * writes dx (fp16 rounded, IN) if dx != NULL. delta scratch: 2*W floats. */
static void mlp_bwd_sample(const mlp_view* v, uint32_t act, const float* x, const float* h, const float* g,
                           float* wgrad, float* dx, float* scratch, float* deltas) {
	const uint32_t W = v->W, IN = v->IN, NH = v->NH, OUTP = v->OUTP;
	if (NH == 0) {  /* dWout[o][k] += g[o] x[k]; dx = Wout^T g */
		const float* Wo = v->wf;
		if (wgrad)
			for (uint32_t o = 0; o < OUTP; ++o) {
				if (g[o] == 0.0f) continue;
				for (uint32_t k = 0; k < IN; ++k) wgrad[(size_t)o * IN + k] += WTERM(g[o] * x[k]);
			}
		if (dx)
			for (uint32_t k = 0; k < IN; ++k) {
				float acc = 0.0f;
				for (uint32_t o = 0; o < OUTP; ++o) acc += DTERM(Wo[(size_t)o * IN + k], g[o]);
				dx[k] = orc_h2f(orc_f2h(acc));
			}
		return;
	}
	float* d_cur = scratch;      /* delta of layer being processed (fp16-rounded) */
	float* d_nxt = scratch + W;
	/* output layer: dWout[o][k] += g[o] * h_last[k]; delta_H = act'(h_H) * Wout^T g */
	const float* Wo = v->wf + v->off[NH];
	const float* hl = h + (size_t)(NH - 1) * W;
	if (wgrad) {
		float* gWo = wgrad + v->off[NH];
		for (uint32_t o = 0; o < OUTP; ++o) {
			if (g[o] == 0.0f) continue;
			for (uint32_t k = 0; k < W; ++k) gWo[(size_t)o * W + k] += WTERM(g[o] * hl[k]);
		}
	}
	for (uint32_t k = 0; k < W; ++k) {
		float acc = 0.0f, part = 0.0f;
		for (uint32_t o = 0; o < OUTP; ++o) { part += DTERM(Wo[(size_t)o * W + k], g[o]); MIMIC_STEP(acc, part, o, 16, OUTP); }
		if (!g_mimic) acc = part;
		d_cur[k] = DABS(act_bwd(act, acc, hl[k]));
	}
	if (deltas) memcpy(deltas + (size_t)(NH - 1) * W, d_cur, sizeof(float) * W);
	/* hidden layers, from the last to the first hidden matmul */
	for (uint32_t l = NH - 1; l >= 1; --l) {
		const float* Wl = v->wf + v->off[l];
		const float* hin = h + (size_t)(l - 1) * W;
		if (wgrad) {
			float* gWl = wgrad + v->off[l];
			for (uint32_t n = 0; n < W; ++n) {
				float dn = d_cur[n];
				if (dn == 0.0f) continue;
				for (uint32_t k = 0; k < W; ++k) gWl[(size_t)n * W + k] += WTERM(dn * hin[k]);
			}
		}
		for (uint32_t k = 0; k < W; ++k) {
			float acc = 0.0f, part = 0.0f;
			for (uint32_t n = 0; n < W; ++n) { part += DTERM(Wl[(size_t)n * W + k], d_cur[n]); MIMIC_STEP(acc, part, n, 16, W); }
			if (!g_mimic) acc = part;
			d_nxt[k] = DABS(act_bwd(act, acc, hin[k]));
		}
		float* t = d_cur; d_cur = d_nxt; d_nxt = t;
		if (deltas) memcpy(deltas + (size_t)(l - 1) * W, d_cur, sizeof(float) * W);
	}
	/* first layer: dW0[n][k] += delta_1[n] * x[k]; dx = W0^T delta_1 */
	const float* W0 = v->wf + v->off[0];
	if (wgrad) {
		float* gW0 = wgrad + v->off[0];
		for (uint32_t n = 0; n < W; ++n) {
			float dn = d_cur[n];
			if (dn == 0.0f) continue;
			for (uint32_t k = 0; k < IN; ++k) gW0[(size_t)n * IN + k] += WTERM(dn * x[k]);
		}
	}
	if (dx) {
		for (uint32_t k = 0; k < IN; ++k) {
			float acc = 0.0f, part = 0.0f;
			for (uint32_t n = 0; n < W; ++n) { part += DTERM(W0[(size_t)n * IN + k], d_cur[n]); MIMIC_STEP(acc, part, n, 8, W); }
			if (!g_mimic) acc = part;
			dx[k] = orc_h2f(orc_f2h(acc));
		}
	}
}

void orc_mlp_bwd(uint32_t W, uint32_t IN, uint32_t NH, uint32_t OUTP, uint32_t act,
                 const uint16_t* params, uint32_t B, const uint16_t* input, int input_soa,
                 const uint16_t* hidden, const uint16_t* dL_dout, float* wgrad,
                 uint16_t* dL_dinput, int n_threads) {
	mlp_view v;
	mlp_view_init(&v, W, IN, NH, OUTP, params);
	size_t np = orc_mlp_n_params(W, IN, NH, OUTP);
	if (n_threads <= 0) n_threads = 1;
	float* partial = (float*)calloc((size_t)n_threads * np, sizeof(float));
	float* deltas = g_mimic ? (float*)malloc(sizeof(float) * (size_t)B * NH * W) : NULL;  /* [B][NH][W] */
#ifdef _OPENMP
#pragma omp parallel num_threads(n_threads)
#endif
	{
		int tid = 0;
#ifdef _OPENMP
		tid = omp_get_thread_num();
#endif
		float* wg = partial + (size_t)tid * np;
		float* x = (float*)malloc(sizeof(float) * IN);
		float* h = (float*)malloc(sizeof(float) * NH * W);
		float* g = (float*)malloc(sizeof(float) * OUTP);
		float* dx = (float*)malloc(sizeof(float) * IN);
		float* scratch = (float*)malloc(sizeof(float) * 2 * W);
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
		for (int64_t ii = 0; ii < (int64_t)B; ++ii) {
			uint32_t i = (uint32_t)ii;
			for (uint32_t k = 0; k < IN; ++k) x[k] = in_at(input, input_soa, IN, B, i, k);
			for (uint32_t l = 0; l < NH; ++l)
				for (uint32_t n = 0; n < W; ++n) h[(size_t)l * W + n] = orc_h2f(hidden[(size_t)l * W * B + (size_t)i * W + n]);
			for (uint32_t o = 0; o < OUTP; ++o) g[o] = orc_h2f(dL_dout[(size_t)i * OUTP + o]);
			mlp_bwd_sample(&v, act, x, h, g, g_mimic ? NULL : wg, dL_dinput ? dx : NULL, scratch,
			               g_mimic ? deltas + (size_t)i * NH * W : NULL);
			if (dL_dinput) {
				for (uint32_t k = 0; k < IN; ++k) {
					uint16_t hv = orc_f2h(dx[k]);
					if (input_soa) dL_dinput[(size_t)k * B + i] = hv; else dL_dinput[(size_t)i * IN + k] = hv;
				}
			}
		}
		free(x); free(h); free(g); free(dx); free(scratch);
	}
	if (g_mimic) {
		/* CUTLASS split-K weight gradients (fully_fused_mlp.cu:775-829): slices of min(4096, B)
		 * samples, each accumulated in fp16 per 8-sample mma step, slice partials summed in fp16 */
		const uint32_t slice = B < 4096 ? B : 4096;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 16) num_threads(n_threads)
#endif
		for (int64_t pp = 0; pp < (int64_t)np; ++pp) {
			const size_t p = (size_t)pp;
			uint32_t m, r, c, K;  /* matrix m (0 = W0, 1..NH-1 hidden, NH = Wout), row r, column c */
			if (p < v.off[1 < NH ? 1 : NH]) { m = 0; K = IN; }
			else if (p >= v.off[NH]) { m = NH; K = W; }
			else { m = 1 + (uint32_t)((p - v.off[1]) / ((size_t)W * W)); K = W; }
			r = (uint32_t)((p - v.off[m]) / K);
			c = (uint32_t)((p - v.off[m]) % K);
			float tot = 0.0f;
			for (uint32_t s0 = 0; s0 < B; s0 += slice) {
				float acc = 0.0f, part = 0.0f;
				for (uint32_t i = s0; i < s0 + slice && i < B; ++i) {
					const float dy = m == NH ? orc_h2f(dL_dout[(size_t)i * OUTP + r]) : deltas[((size_t)i * NH + m) * W + r];
					const float xv = m == 0 ? in_at(input, input_soa, IN, B, i, c)
					                        : orc_h2f(hidden[(size_t)(m - 1) * W * B + (size_t)i * W + c]);
					part += dy * xv;
					MIMIC_STEP(acc, part, i - s0, 8, slice);
				}
				tot = hround(tot + acc);
			}
			wgrad[p] = tot;
		}
		free(deltas);
	} else {
		for (size_t p = 0; p < np; ++p) {
			float s = 0.0f;
			for (int t = 0; t < n_threads; ++t) s += partial[(size_t)t * np + p];
			wgrad[p] = s;
		}
	}
	free(partial);
	free(v.wf);
}

/* ------------------------------------------------------------------------------------------ */
/* OneBlob -- encodings/oneblob.h:46-164, quartic_cdf common_device.h:905-920                  */
/* ------------------------------------------------------------------------------------------ */
/* nvcc compiles the reference with FMA contraction on; the contracted forms are written out. */
static uint32_t orc_log2u(uint32_t v) { /* (uint32_t)std::log2(n_bins) for powers of two */
	uint32_t r = 0;
	while ((1u << r) < v) ++r;
	return r;
}
static float quartic_cdf(float x, float inv_radius) {
	const float u = x * inv_radius;
	const float u2 = u * u;
	const float u4 = u2 * u2;
	float p = fmaf(-(2.0f / 3.0f), u2, 1.0f);
	p = fmaf(1.0f / 5.0f, u4, p);
	return fmaxf(0.0f, fminf(1.0f, fmaf((15.0f / 16.0f) * u, p, 0.5f)));
}
static float quartic_cdf_deriv(float x, float inv_radius) {
	const float u = x * inv_radius;
	const float tmp = fmaxf(fmaf(-u, u, 1.0f), 0.0f);
	return (15.0f / 16.0f) * tmp * tmp * inv_radius;
}
/* left-boundary CDF with wrap-around (one_blob_subwarp_aligned, oneblob.h:48-51) */
static float oneblob_left_cdf(uint32_t bin, uint32_t n_bins, float x) {
	const float d = ldexpf((float)bin, -(int)orc_log2u(n_bins)) - x;
	return quartic_cdf(d, (float)n_bins) + quartic_cdf(d - 1.0f, (float)n_bins) + quartic_cdf(d + 1.0f, (float)n_bins);
}

void orc_oneblob_fwd(uint32_t B, uint32_t D, uint32_t n_bins, const float* x, uint16_t* out, uint32_t stride, uint32_t n_pad) {
	/* Reference lane j (= encoded index) holds bin b = j & (n_bins-1); the right CDF comes from
	 * __shfl_sync(mask, left, b + 1, n_bins) (oneblob.h:57). The shuffle width is clamped by the 32-lane
	 * warp: the source is lane ((b + 1) mod S) of the lane's S-wide segment, S = min(n_bins, 32), so
	 * for n_bins = 64 bin 31 reads bin 0's left CDF and bin 63 reads bin 32's (+1 at the last bin). */
	const uint32_t S = n_bins < 32 ? n_bins : 32;
	for (uint32_t i = 0; i < B; ++i) {
		uint16_t* row = out + (size_t)i * stride;
		for (uint32_t d = 0; d < D; ++d) {
			const float xv = x[(size_t)i * D + d];
			for (uint32_t b = 0; b < n_bins; ++b) {
				const uint32_t src = (b & ~(S - 1)) + ((b + 1) & (S - 1));
				float right = oneblob_left_cdf(src, n_bins, xv);
				if (b == n_bins - 1) right += 1.0f;
				row[d * n_bins + b] = orc_f2h(right - oneblob_left_cdf(b, n_bins, xv));
			}
		}
		for (uint32_t j = 0; j < n_pad; ++j) row[D * n_bins + j] = orc_f2h(1.0f);
	}
}

void orc_oneblob_bwd(uint32_t B, uint32_t D, uint32_t n_bins, const float* x, const uint16_t* dy, uint32_t stride, float* dx) {
	const float nb = (float)n_bins;
	for (uint32_t i = 0; i < B; ++i)
		for (uint32_t d = 0; d < D; ++d) {
			const float xv = x[(size_t)i * D + d];
			float left = quartic_cdf_deriv(-xv, nb) + quartic_cdf_deriv(-xv - 1.0f, nb) + quartic_cdf_deriv(-xv + 1.0f, nb);
			float result = 0.0f;
			for (uint32_t k = 0; k < n_bins; ++k) {
				const float rb = ldexpf((float)(k + 1), -(int)orc_log2u(n_bins));
				const float right = quartic_cdf_deriv(rb - xv, nb) + quartic_cdf_deriv(rb - xv - 1.0f, nb) + quartic_cdf_deriv(rb - xv + 1.0f, nb);
				const float deriv = left - right;
				left = right;
				result = fmaf(orc_h2f(dy[(size_t)i * stride + d * n_bins + k]), deriv, result);
			}
			dx[(size_t)i * D + d] = result;
		}
}

void orc_identity_fwd(uint32_t B, uint32_t D, float scale, float offset, const float* x, uint16_t* out, uint32_t stride,
                      uint32_t n_pad) {
	for (uint32_t i = 0; i < B; ++i)
		for (uint32_t j = 0; j < D + n_pad; ++j)
			out[(size_t)i * stride + j] = orc_f2h(j < D ? fmaf(x[(size_t)i * D + j], scale, offset) : 1.0f);
}

/* ------------------------------------------------------------------------------------------ */
/* RelativeL2 -- losses/relative_l2.h:40-76                                                     */
/* ------------------------------------------------------------------------------------------ */
double orc_relative_l2(uint32_t B, uint32_t stride, uint32_t dims, float loss_scale,
                       const uint16_t* pred, const float* target, float* values, uint16_t* grads) {
	const uint32_t n_elements = B * stride;
	const uint32_t n_total = n_elements / stride * dims;
	double sum = 0.0;
	for (uint32_t i = 0; i < n_elements; ++i) {
		uint32_t intra = i % stride, inter = i / stride;
		if (intra >= dims) {
			if (values) values[i] = 0.0f;
			grads[i] = 0;
			continue;
		}
		uint32_t ti = inter * dims + intra;
		float p = orc_h2f(pred[i]);
		float pse = fmaf(p, p, 0.01f);
		float d = p - target[ti];
		float val = d * d / pse / 1.0f / (float)n_total;
		float gr = 2.0f * d / pse / 1.0f;
		if (values) values[i] = val;
		sum += val;
		grads[i] = orc_f2h(loss_scale * gr / (float)n_total);
	}
	return sum;
}

/* L2 -- losses/l2.h:40-76 (data_pdf = 1) */
double orc_l2(uint32_t B, uint32_t stride, uint32_t dims, float loss_scale,
              const uint16_t* pred, const float* target, float* values, uint16_t* grads) {
	const uint32_t n_elements = B * stride;
	const uint32_t n_total = n_elements / stride * dims;
	double sum = 0.0;
	for (uint32_t i = 0; i < n_elements; ++i) {
		uint32_t intra = i % stride, inter = i / stride;
		if (intra >= dims) {
			if (values) values[i] = 0.0f;
			grads[i] = 0;
			continue;
		}
		uint32_t ti = inter * dims + intra;
		float d = orc_h2f(pred[i]) - target[ti];
		float val = d * d / 1.0f / (float)n_total;
		float gr = 2.0f * d / 1.0f;
		if (values) values[i] = val;
		sum += val;
		grads[i] = orc_f2h(loss_scale * gr / (float)n_total);
	}
	return sum;
}

/* ------------------------------------------------------------------------------------------ */
/* Adam -- optimizers/adam.h:47-188                                                            */
/* ------------------------------------------------------------------------------------------ */
void orc_adam_default(orc_adam_cfg* c) { /* adam.h:309-325 */
	c->learning_rate = 1e-3f; c->beta1 = 0.9f; c->beta2 = 0.999f; c->epsilon = 1e-8f; c->l2_reg = 1e-8f;
	c->relative_decay = 0.0f; c->absolute_decay = 0.0f; c->clipping_magnitude = 0.0f;
	c->non_matrix_learning_rate_factor = 1.0f;
	c->adabound = 0; c->optimize_matrix_params = 1; c->optimize_non_matrix_params = 1;
}

void orc_adam_step(const orc_adam_cfg* c, uint32_t n, uint32_t n_matrix, float loss_scale,
                   uint32_t current_step, float* w32, uint16_t* w16, const uint16_t* grad16,
                   float* m1, float* m2, uint32_t* steps) {
	float lower = 0.0f, upper = 3.402823466e+38f;
	if (c->adabound) { /* adam.h:156-159 */
		lower = 0.1f - 0.1f / ((1 - c->beta2) * (float)current_step + 1);
		upper = 0.1f + 0.1f / ((1 - c->beta2) * (float)current_step);
	}
	for (uint32_t i = 0; i < n; ++i) {
		float gradient = orc_h2f(grad16[i]) / loss_scale;
		if (i >= n_matrix) {
			if (!c->optimize_non_matrix_params || gradient == 0) continue;
		} else {
			if (!c->optimize_matrix_params) continue;
		}
		const float wfp = w32[i];
		if (i < n_matrix) gradient = fmaf(c->l2_reg, wfp, gradient);
		const float gsq = gradient * gradient;
		const float mm1 = m1[i] = fmaf(c->beta1, m1[i], (1 - c->beta1) * gradient);
		const float mm2 = m2[i] = fmaf(c->beta2, m2[i], (1 - c->beta2) * gsq);
		float lr = c->learning_rate;
		if (i >= n_matrix) lr *= c->non_matrix_learning_rate_factor;
		const uint32_t st = ++steps[i];
		lr *= sqrtf(1 - powf(c->beta2, (float)st)) / (1 - powf(c->beta1, (float)st));
		const float eff = fminf(fmaxf(lr / (sqrtf(mm2) + c->epsilon), lower), upper);
		/* weight_decay, common_device.h:870-873 */
		const float decayed = fmaf(1 - c->relative_decay * lr, wfp, -copysignf(c->absolute_decay * lr, wfp));
		float nw = fmaf(-eff, mm1, decayed);
		if (c->clipping_magnitude != 0.0f) {
			nw = fminf(fmaxf(nw, -c->clipping_magnitude), c->clipping_magnitude);
		}
		w32[i] = nw;
		w16[i] = orc_f2h(nw);
	}
}

/* ------------------------------------------------------------------------------------------ */
/* Trainer (trainer.h:50-190) for NetworkWithInputEncoding<Grid, FullyFusedMLP>                  */
/* ------------------------------------------------------------------------------------------ */

static uint32_t model_enc_params(const orc_model* m) { return m->enc_type == 0 ? m->grid.n_params : 0u; }

/* encoding forward: grid -> SoA [IN][B] (returns 1), OneBlob / Identity -> AoS [B][IN] (returns 0) */
static int model_encode(const orc_model* m, uint32_t B, const float* pos, uint16_t* enc) {
	if (m->enc_type == 1) {
		orc_oneblob_fwd(B, m->n_dims, m->n_bins, pos, enc, m->IN, m->IN - m->n_dims * m->n_bins);
		return 0;
	}
	if (m->enc_type == 2) {
		orc_identity_fwd(B, m->n_dims, m->enc_scale, m->enc_offset, pos, enc, m->IN, m->IN - m->n_dims);
		return 0;
	}
	orc_grid_fwd(&m->grid, B, pos, m->w16 + m->n_mlp_params, enc);
	return 1;
}

int orc_model_init(orc_model* m, uint32_t seed) {
	if (m->enc_type == 0) {
		if (orc_grid_init(&m->grid) != 0) return -1;
		m->IN = m->grid.n_levels * m->grid.n_features_per_level;
	}
	const uint32_t IN = m->IN;
	m->n_mlp_params = orc_mlp_n_params(m->W, IN, m->NH, m->OUTP);
	m->n_params = m->n_mlp_params + model_enc_params(m);
	m->adam_step = 0;
	size_t n = m->n_params;
	m->w32 = (float*)calloc(n, 4); m->w16 = (uint16_t*)calloc(n, 2);
	m->grad16 = (uint16_t*)calloc(n, 2); m->grad32 = (float*)calloc(n, 4);
	m->m1 = (float*)calloc(n, 4); m->m2 = (float*)calloc(n, 4); m->steps = (uint32_t*)calloc(n, 4);
	/* trainer.h:52-55: rng = pcg32{seed_seq{seed}[0]} */
	uint32_t s[2];
	orc_seed_seq(&seed, 1, s, 2);
	orc_pcg32 rng;
	orc_pcg32_seed(&rng, s[0], 1u);
	/* NWIE::initialize_params (network_with_input_encoding.h:124-130): network first */
	float* p = m->w32;
	if (m->NH == 0) {  /* CutlassMLP with no hidden layer: one matrix */
		orc_xavier_uniform(&rng, m->OUTP, IN, p, 1.0f); p += (size_t)m->OUTP * IN;
	} else {
		orc_xavier_uniform(&rng, m->W, IN, p, 1.0f); p += (size_t)m->W * IN;
		for (uint32_t k = 1; k < m->NH; ++k) { orc_xavier_uniform(&rng, m->W, m->W, p, 1.0f); p += (size_t)m->W * m->W; }
		orc_xavier_uniform(&rng, m->OUTP, m->W, p, 1.0f); p += (size_t)m->OUTP * m->W;
	}
	/* GridEncodingTemplated::initialize_params (grid.h:1059-1062) */
	if (m->enc_type == 0) orc_generate_uniform(&rng, m->grid.n_params, p, -1e-4f, 1e-4f);
	orc_f2h_array(m->w32, m->w16, n); /* trainer.h:83-85 */
	return 0;
}

void orc_model_free(orc_model* m) {
	free(m->w32); free(m->w16); free(m->grad16); free(m->grad32); free(m->m1); free(m->m2); free(m->steps);
	memset(m, 0, sizeof(*m));
}

void orc_model_inference(orc_model* m, uint32_t B, const float* pos, uint16_t* out, int n_threads) {
	const uint32_t IN = m->IN;
	uint16_t* enc = (uint16_t*)malloc((size_t)IN * B * 2);
	const int soa = model_encode(m, B, pos, enc);
	orc_mlp_fwd(m->W, IN, m->NH, m->OUTP, m->activation, m->w16, B, enc, soa, out, NULL, n_threads);
	free(enc);
}

double orc_train_step(orc_model* m, uint32_t B, const float* pos, const float* target, int run_optimizer, int n_threads) {
	const uint32_t IN = m->IN;
	const float loss_scale = 128.0f; /* default_loss_scale<__half> (common.h:232) */
	uint16_t* enc = (uint16_t*)malloc((size_t)IN * B * 2);
	uint16_t* out = (uint16_t*)malloc((size_t)m->OUTP * B * 2);
	uint16_t* hidden = (uint16_t*)malloc((size_t)m->NH * m->W * B * 2);
	uint16_t* dout = (uint16_t*)malloc((size_t)m->OUTP * B * 2);
	uint16_t* denc = (uint16_t*)malloc((size_t)IN * B * 2);
	const int soa = model_encode(m, B, pos, enc);
	orc_mlp_fwd(m->W, IN, m->NH, m->OUTP, m->activation, m->w16, B, enc, soa, out, hidden, n_threads);
	double loss = m->loss_type == 1 ? orc_l2(B, m->OUTP, m->n_output_dims, loss_scale, out, target, NULL, dout)
	                                : orc_relative_l2(B, m->OUTP, m->n_output_dims, loss_scale, out, target, NULL, dout);
	/* output-activation transfer of dL/dout (fully_fused_mlp.cu:759-762, activation_backward_output_gpu) */
	orc_act_bwd_output(m->activation, (size_t)m->OUTP * B, out, dout);
	orc_mlp_bwd(m->W, IN, m->NH, m->OUTP, m->activation, m->w16, B, enc, soa, hidden, dout, m->grad32,
	            m->enc_type == 0 ? denc : NULL, n_threads);
	if (m->enc_type == 0) {
		memset(m->grad32 + m->n_mlp_params, 0, (size_t)m->grid.n_params * 4);
		orc_grid_bwd(&m->grid, B, pos, denc, m->grad32 + m->n_mlp_params);
	}
	orc_f2h_array(m->grad32, m->grad16, m->n_params);
	if (run_optimizer) {
		m->adam_step++;
		orc_adam_step(&m->adam, m->n_params, m->n_mlp_params, loss_scale, m->adam_step,
		              m->w32, m->w16, m->grad16, m->m1, m->m2, m->steps);
	}
	free(enc); free(out); free(hidden); free(dout); free(denc);
	return loss;
}
