// grid_bwd_lds.h -- the LDS-privatised grid backward (reference kernel_grid_backward, grid.h:214-320):
// kernel template and per-D launchers, instantiated once per input dimension in grid_bwd_d{2,3,4}.hip
// (one translation unit per D keeps the parallel build short).
#pragma once

#include "kernels.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "adam_device.h"
#include "grid_device.h"

namespace tcnn_amd {

// LDS accumulators are int32 fixed point with a per-(work item, chunk) power-of-two scale.
// gfx950 executes LDS float atomics (ds_add_f32 / ds_pk_add_f16) at ~195 cycles per wave-instruction
// per CU but ds_add_u32 at ~8 (tools/lds_atomic_bench.hip), and integer sums are order-independent,
// so the gradient is bit-reproducible (the reference's fp16 atomics, grid.h:252-255, are not).
// Range: the bilinear weights of one point sum to 1, so no table entry can receive more than
// sum_i |dL/dy_i| over a chunk's points (hash collisions included); the scale 2^e is the largest
// power of two that keeps that bound plus the rounding of every add below 2^31, i.e. one add
// resolves 2^-31 * sum |dL/dy| ~ 2^-16 * mean |dL/dy| for the ~2^15-point chunks of B = 2^18
// (finer than the reference's fp16 running sums, and insensitive to a single outlier dL/dy).
// 32-bit accumulators let a whole 32768-entry hashed level (one feature) or a whole dense level
// (all features) sit in 128 KiB of LDS: every corner update lands and no lane is masked off.
// Levels larger than that take the binned backward (grid_bin.hip).
constexpr uint32_t GRID_BWD_THREADS = 1024;
constexpr uint32_t GRID_BWD_LDS_BYTES = 128 * 1024;
constexpr uint32_t GRID_BWD_SLOTS = GRID_BWD_LDS_BYTES / 4;



__device__ __forceinline__ void lds_add_i32(int* acc, float v) {
	__hip_atomic_fetch_add(acc, __float2int_rn(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Index kinds of a level, uniform per work item (reference grid_index, common_device.h:690-707):
//   HASH_POW2  hashed level of power-of-two size: index = hash & (size - 1)
//   DENSE      res^D <= size: index = sum g_d res^d, < 2 size, so `% size` is one conditional subtract
//   GENERIC    anything else (tiled grids, non-power-of-two hashed sizes): grid_index()
//   HASH_RANGE a contiguous entry range [begin, begin + len) of such a hashed level (r06: a hashed
//              level too large for the LDS is split into entry ranges holding all F features, so its
//              slab is in parameter order; corners outside the range are skipped)
enum : int { IDX_HASH_POW2 = 0, IDX_DENSE = 1, IDX_GENERIC = 2, IDX_HASH_RANGE = 3 };

template <uint32_t D, HashType H, int KIND>
__device__ __forceinline__ uint32_t level_index(bool hash_grid, uint32_t size, uint32_t res, const uint32_t* g) {
	if constexpr (KIND == IDX_HASH_POW2 || KIND == IDX_HASH_RANGE) {
		uint32_t h = 0;
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) h ^= g[d] * hash_prime<H>(d);
		return h & (size - 1);
	} else if constexpr (KIND == IDX_DENSE) {
		uint32_t idx = 0, stride = 1;
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) {
			idx += g[d] * stride;
			stride *= res;
		}
		// index % size (common_device.h:706): in-range positions give idx < 2 size; positions
		// outside [0, 1] can give any value
		if (idx >= size) {
			idx -= size;
			if (idx >= size) idx %= size;
		}
		return idx;
	} else {
		return grid_index<D, H>(hash_grid, size, res, g);
	}
}

// One point's corner updates of one work item into the LDS accumulators (reference
// kernel_grid_backward's per-level body, grid.h:246-317): dy = the point's dL/dy already multiplied by
// the item's fixed-point scale.
template <uint32_t D, uint32_t F, HashType H, int KIND, int MODE, bool OPTS>
__device__ __forceinline__ void accum_point(const float (&x)[D], const float (&dy)[F], uint32_t i, uint32_t level, uint32_t B,
                                            const LevelInfo& li, bool hash_grid, Interp interp, uint32_t begin, uint32_t len,
                                            uint32_t f0, uint32_t nf, int* acc, const GridOpts& o) {
	float p[D];
	uint32_t pg[D];
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) pos_fract(x[d], li.scale, interp, p[d], pg[d]);
	const bool nearest = interp == Interp::Nearest;
	// stochastic interpolation (grid.h:284-298): one corner, chosen per (point, level), weight 1
	const bool single = nearest || (OPTS && o.stochastic);
	uint32_t cbits = 0;
	if (single && !nearest) {
		const float smp = random_val_1337(i + level * B);
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) cbits |= (smp >= p[d] ? 0u : 1u) << d;
	}
#pragma unroll
	for (uint32_t c0 = 0; c0 < (1u << D); ++c0) {
		if (single && c0 > 0) break;
		const uint32_t c = single ? cbits : c0;
		float w = 1.0f;
		uint32_t local[D];
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) {
			if ((c & (1u << d)) == 0) { w *= 1.0f - p[d]; local[d] = pg[d]; }
			else { w *= p[d]; local[d] = pg[d] + 1; }
		}
		const float wh = single ? 1.0f : (float)f16_rn(w);
		const uint32_t rel = level_index<D, H, KIND>(hash_grid, li.size, li.res, local) - begin;
		if constexpr (KIND == IDX_GENERIC || KIND == IDX_HASH_RANGE) {  // entry slices may not cover the level
			if (rel >= len) continue;
		}
		if constexpr (MODE == 0) {
			const int a = __float2int_rn(wh * dy[0]);
			const int b = __float2int_rn(wh * dy[1]);
			const unsigned long long pk = (unsigned long long)(((long long)b << 32) + (long long)a);
			__hip_atomic_fetch_add((unsigned long long*)acc + rel, pk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
		} else {
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) {
				if constexpr (MODE == 1) {
					if (f - f0 < nf) lds_add_i32(&acc[rel * nf + (f - f0)], wh * dy[f]);
				} else {
					lds_add_i32(&acc[rel * F + f], wh * dy[f]);
				}
			}
		}
	}
}

// One point's corner updates, D == 2, Linear interpolation, a whole level of kind HASH_POW2 or
// DENSE (for DENSE: a position in [0, 1], so every corner index is below 2 size) -- accum_point's
// arithmetic with the per-dimension hash / dense terms computed once per point and no control flow
// per corner. (As generic code the per-corner index and `% size` paths became exec-mask branches
// around every corner, as in the fused kernel's encode, r03.)
template <uint32_t F, HashType H, int KIND, int MODE>
__device__ __forceinline__ void accum_point_2d_fast(const float (&x)[2], const float (&dy)[F], const LevelInfo& li, uint32_t f0,
                                                    uint32_t nf, int* acc, uint32_t begin = 0, uint32_t len = 0) {
	float p[2];
	uint32_t g[2];
	pos_fract(x[0], li.scale, Interp::Linear, p[0], g[0]);
	pos_fract(x[1], li.scale, Interp::Linear, p[1], g[1]);
	uint32_t t[2][2];
	if constexpr (KIND == IDX_HASH_POW2 || KIND == IDX_HASH_RANGE) {
		t[0][0] = g[0] * hash_prime<H>(0);
		t[0][1] = t[0][0] + hash_prime<H>(0);
		t[1][0] = g[1] * hash_prime<H>(1);
		t[1][1] = t[1][0] + hash_prime<H>(1);
	} else {
		t[0][0] = g[0];
		t[0][1] = g[0] + 1u;
		t[1][0] = g[1] * li.res;
		t[1][1] = t[1][0] + li.res;
	}
#pragma unroll
	for (uint32_t c = 0; c < 4; ++c) {
		const uint32_t bx = c & 1u, by = c >> 1;
		const float w = (bx ? p[0] : 1.0f - p[0]) * (by ? p[1] : 1.0f - p[1]);
		const float wh = (float)f16_rn(w);
		uint32_t rel;
		if constexpr (KIND == IDX_HASH_POW2) {
			rel = (t[0][bx] ^ t[1][by]) & (li.size - 1u);
		} else if constexpr (KIND == IDX_HASH_RANGE) {
			rel = ((t[0][bx] ^ t[1][by]) & (li.size - 1u)) - begin;
			if (rel >= len) continue;  // another range's corner (exec-masked, no branch around the point)
		} else {
			const uint32_t d = t[0][bx] + t[1][by];
			rel = __builtin_elementwise_min(d, d - li.size);  // d % size for d < 2 size
		}
		if constexpr (MODE == 0) {
			const int a = __float2int_rn(wh * dy[0]);
			const int b = __float2int_rn(wh * dy[1]);
			const unsigned long long pk = (unsigned long long)(((long long)b << 32) + (long long)a);
			__hip_atomic_fetch_add((unsigned long long*)acc + rel, pk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
		} else {
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) {
				if constexpr (MODE == 1) {
					if (f - f0 < nf) lds_add_i32(&acc[rel * nf + (f - f0)], wh * dy[f]);
				} else {
					lds_add_i32(&acc[rel * F + f], wh * dy[f]);
				}
			}
		}
	}
}

// Register-resident variant (D == 2, F <= 2, no grid options): the chunk's dL/dy bits were loaded
// into dyb (GRID_BWD_PR points per thread, point i0 + threadIdx.x + p * blockDim.x in slot p) for the
// scale pre-pass and are reused here; positions stream in batches of 8 with the next batch in flight.
constexpr uint32_t GRID_BWD_PR = 32, GRID_BWD_PU = 8;
static_assert(GRID_BWD_THREADS * GRID_BWD_PR == GRID_BWD_REG_POINTS, "kernels.h GRID_BWD_REG_POINTS");
template <uint32_t D>
__device__ __forceinline__ void load_pos_batch(const float* __restrict__ pos, uint32_t pstride, uint32_t i0, uint32_t i1, uint32_t k,
                                               float (&dst)[GRID_BWD_PU][D]) {
#pragma unroll
	for (uint32_t u = 0; u < GRID_BWD_PU; ++u) {
		const uint32_t i = i0 + threadIdx.x + (k * GRID_BWD_PU + u) * blockDim.x;
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) dst[u][d] = i < i1 ? pos[(size_t)i * pstride + d] : 0.0f;
	}
}

template <uint32_t D, uint32_t F, HashType H, int KIND, int MODE>
__device__ __forceinline__ void grid_bwd_points_regs(const uint32_t (&dyb)[GRID_BWD_PR], const float (&xs0)[GRID_BWD_PU][D],
                                                     uint32_t B, const float* __restrict__ pos,
                                                     uint32_t pstride, uint32_t level, const LevelInfo& li, bool hash_grid,
                                                     Interp interp, uint32_t begin, uint32_t len, uint32_t f0, uint32_t nf,
                                                     uint32_t i0, uint32_t i1, float scale, int* acc, const GridOpts& o) {
	constexpr uint32_t U = GRID_BWD_PU, NB = GRID_BWD_PR / U;
	constexpr bool FAST_KIND = D == 2 && (KIND == IDX_HASH_POW2 || KIND == IDX_DENSE || KIND == IDX_HASH_RANGE);
	const bool fast = FAST_KIND && interp == Interp::Linear && (begin == 0 || KIND == IDX_HASH_RANGE);  // whole levels or hash ranges
	float xs[2][U][D];
#pragma unroll
	for (uint32_t u = 0; u < U; ++u)
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) xs[0][u][d] = xs0[u][d];
#pragma unroll
	for (uint32_t k = 0; k < NB; ++k) {
		if (i0 + threadIdx.x + k * U * blockDim.x >= i1) break;
		if (k + 1 < NB) load_pos_batch<D>(pos, pstride, i0, i1, k + 1, xs[(k + 1) & 1]);
		bool fast_b = fast;
		if constexpr (FAST_KIND && KIND == IDX_DENSE) {  // dense corners below 2 size need positions in [0, 1]
			bool inr = true;
#pragma unroll
			for (uint32_t u = 0; u < U; ++u)
#pragma unroll
				for (uint32_t d = 0; d < D; ++d) inr = inr && xs[k & 1][u][d] >= 0.0f && xs[k & 1][u][d] <= 1.0f;
			fast_b = fast_b && __builtin_amdgcn_ballot_w64(!inr) == 0;
		}
		if (fast_b) {
			if constexpr (FAST_KIND) {
				if (i0 + threadIdx.x + (k * U + U - 1) * blockDim.x < i1) {  // the whole batch is inside the chunk
#pragma unroll
					for (uint32_t u = 0; u < U; ++u) {
						const uint32_t p = k * U + u;
						float dy[F];
#pragma unroll
						for (uint32_t f = 0; f < F; ++f) dy[f] = dy_bits_feature(dyb[p], f) * scale;
						accum_point_2d_fast<F, H, KIND, MODE>(*(const float(*)[2]) & xs[k & 1][u][0], dy, li, f0, nf, acc, begin, len);
					}
				} else {
					// the chunk's last, partial batch (e.g. 4 points per thread at 4096-point chunks: the
					// 2^15-point shard of N = 8): the same branch-free path per point that exists (r04 sent
					// these through the generic per-corner path, 3.5 us of accumulation for 4 points)
#pragma unroll
					for (uint32_t u = 0; u < U; ++u) {
						const uint32_t p = k * U + u;
						if (i0 + threadIdx.x + p * blockDim.x >= i1) break;
						float dy[F];
#pragma unroll
						for (uint32_t f = 0; f < F; ++f) dy[f] = dy_bits_feature(dyb[p], f) * scale;
						accum_point_2d_fast<F, H, KIND, MODE>(*(const float(*)[2]) & xs[k & 1][u][0], dy, li, f0, nf, acc, begin, len);
					}
				}
			}
			continue;
		}
#pragma unroll
		for (uint32_t u = 0; u < U; ++u) {
			const uint32_t p = k * U + u;
			const uint32_t i = i0 + threadIdx.x + p * blockDim.x;
			if (i >= i1) break;
			float dy[F];
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) dy[f] = dy_bits_feature(dyb[p], f) * scale;
			accum_point<D, F, H, KIND, MODE, false>(xs[k & 1][u], dy, i, level, B, li, hash_grid, interp, begin, len, f0, nf, acc, o);
		}
	}
}

// MODE: 0 = F == 2, both features as one packed int64 (two int32 halves) per entry -> one
// ds_add_u64 per corner; 1 = the feature group [f0, f0 + nf) per entry (nf < F), ds_add_u32;
// 2 = all F features, ds_add_u32.
template <uint32_t D, uint32_t F, HashType H, int KIND, int MODE, bool OPTS>
__device__ __forceinline__ void grid_bwd_points(int layout, uint32_t B, const float* __restrict__ pos, uint32_t pstride,
                                                const _Float16* __restrict__ dLdy, uint32_t dy_stride, uint32_t level,
                                                const LevelInfo& li, bool hash_grid, Interp interp, uint32_t begin,
                                                uint32_t len, uint32_t f0, uint32_t nf, uint32_t i0, uint32_t i1, float scale,
                                                int* acc, const GridOpts& o) {
	constexpr uint32_t NF = F;
	constexpr uint32_t U = 8;  // points in flight per thread
	constexpr bool FAST_KIND = D == 2 && !OPTS && (KIND == IDX_HASH_POW2 || KIND == IDX_DENSE || KIND == IDX_HASH_RANGE);
	const bool fast = FAST_KIND && interp == Interp::Linear && (begin == 0 || KIND == IDX_HASH_RANGE);  // accum_point_2d_fast
	for (uint32_t base = i0 + threadIdx.x; base < i1; base += U * blockDim.x) {
		float xs[U][D], dy[U][NF];
#pragma unroll
		for (uint32_t u = 0; u < U; ++u) {
			const uint32_t i = base + u * blockDim.x;
			float v[F];
			if (i < i1) {
#pragma unroll
				for (uint32_t d = 0; d < D; ++d) xs[u][d] = pos[(size_t)i * pstride + d];
				load_dy<F>(layout, dLdy, dy_stride, level, B, i, v);
			} else {
#pragma unroll
				for (uint32_t d = 0; d < D; ++d) xs[u][d] = 0.0f;
#pragma unroll
				for (uint32_t f = 0; f < F; ++f) v[f] = 0.0f;
			}
			if (OPTS && i < i1 && (float)level > grid_max_level(o, i, F) + 1e-3f) {  // masked (grid.h:242-244)
#pragma unroll
				for (uint32_t f = 0; f < F; ++f) v[f] = 0.0f;
			}
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) dy[u][f] = v[f] * scale;
		}
		if constexpr (FAST_KIND) {
			bool fast_b = fast;
			if constexpr (KIND == IDX_DENSE) {
				bool inr = true;
#pragma unroll
				for (uint32_t u = 0; u < U; ++u)
#pragma unroll
					for (uint32_t d = 0; d < D; ++d) inr = inr && xs[u][d] >= 0.0f && xs[u][d] <= 1.0f;
				fast_b = fast_b && __builtin_amdgcn_ballot_w64(!inr) == 0;
			}
			if (fast_b && base + (U - 1) * blockDim.x < i1) {
#pragma unroll
				for (uint32_t u = 0; u < U; ++u)
					accum_point_2d_fast<F, H, KIND, MODE>(*(const float(*)[2]) & xs[u][0], dy[u], li, f0, nf, acc, begin, len);
				continue;
			}
		}
#pragma unroll
		for (uint32_t u = 0; u < U; ++u) {
			if (base + u * blockDim.x >= i1) break;
			accum_point<D, F, H, KIND, MODE, OPTS>(xs[u], dy[u], base + u * blockDim.x, level, B, li, hash_grid, interp, begin, len, f0,
			                                       nf, acc, o);
		}
	}
}

template <uint32_t D, uint32_t F, HashType H, int KIND, bool OPTS>
__device__ __forceinline__ void grid_bwd_mode(int mode, int layout, uint32_t B, const float* pos, uint32_t pstride,
                                              const _Float16* dLdy, uint32_t dy_stride, uint32_t level, const LevelInfo& li,
                                              bool hash_grid, Interp interp, uint32_t begin, uint32_t len, uint32_t f0,
                                              uint32_t nf, uint32_t i0, uint32_t i1, float scale, int* acc, const GridOpts& o) {
	if constexpr (F == 2) {
		if (mode == 0) { grid_bwd_points<D, F, H, KIND, 0, OPTS>(layout, B, pos, pstride, dLdy, dy_stride, level, li, hash_grid, interp, begin, len, f0, nf, i0, i1, scale, acc, o); return; }
	} else if constexpr (F > 2) {
		if (mode == 2) { grid_bwd_points<D, F, H, KIND, 2, OPTS>(layout, B, pos, pstride, dLdy, dy_stride, level, li, hash_grid, interp, begin, len, f0, nf, i0, i1, scale, acc, o); return; }
	}
	grid_bwd_points<D, F, H, KIND, 1, OPTS>(layout, B, pos, pstride, dLdy, dy_stride, level, li, hash_grid, interp, begin, len, f0, nf, i0, i1, scale, acc, o);
}

template <uint32_t D, uint32_t F, HashType H, int KIND>
__device__ __forceinline__ void grid_bwd_mode_regs(int mode, const uint32_t (&dyb)[GRID_BWD_PR], const float (&xs0)[GRID_BWD_PU][D],
                                                   uint32_t B, const float* pos,
                                                   uint32_t pstride, uint32_t level, const LevelInfo& li, bool hash_grid, Interp interp,
                                                   uint32_t begin, uint32_t len, uint32_t f0, uint32_t nf, uint32_t i0, uint32_t i1,
                                                   float scale, int* acc, const GridOpts& o) {
	if constexpr (F == 2) {
		if (mode == 0) { grid_bwd_points_regs<D, F, H, KIND, 0>(dyb, xs0, B, pos, pstride, level, li, hash_grid, interp, begin, len, f0, nf, i0, i1, scale, acc, o); return; }
	}
	grid_bwd_points_regs<D, F, H, KIND, 1>(dyb, xs0, B, pos, pstride, level, li, hash_grid, interp, begin, len, f0, nf, i0, i1, scale, acc, o);
}

// Network-gradient tail (extra workgroups g = 0 .. n_mlp_groups-1, on CUs the grid items leave
// free): workgroup g sums the fused kernel's slabs for its block of network-parameter columns
// (block_column_sums: the same order as launch_column_sums of the sequential path), applies Adam
// to those parameters and writes them into the next step's fused weight image. No cross-workgroup
// dependency. Workgroup 0 also sums the loss partials and publishes the bias-correction factor.
__device__ __forceinline__ void grid_bwd_mlp_tail(const GridBwdEpilogue& ep, uint32_t g, float* lds) {
	const uint32_t N = ep.n_mlp;
	const uint32_t cb = column_block(N, ep.n_mlp_groups);
	const uint32_t c0 = g * cb;
	if (c0 < N) {
		const uint32_t ncol = min(cb, N - c0);
		float* out = lds;
		float* tmp = lds + cb;
		block_column_sums(ep.wpart, ep.n_wparts, N, c0, ncol, tmp, out);
		const uint32_t nW0 = ep.W * ep.IN, nWh = (ep.NH - 1) * ep.W * ep.W;
		for (uint32_t t = threadIdx.x; t < ncol; t += blockDim.x) {
			const uint32_t i = c0 + t;
			const float s = out[t];
			if (ep.fin.out) {
				grad_finalize_store(s, ep.fin.s, ep.fin.out, i, ep.fin.out_f32);
				continue;
			}
			ep.buf.g32[i] = s;
			if (!ep.apply_adam) continue;
			const _Float16 h = adam_update(ep.adam_mlp, ep.buf, i, s);
			uint32_t o;
			if (i < nW0) {
				o = (i / ep.IN) * ep.RSI + i % ep.IN;
			} else if (i < nW0 + nWh) {
				const uint32_t k = i - nW0;
				o = ep.oWh + (k / ep.W) * ep.RSW + k % ep.W;  // rows of all hidden matrices are consecutive
			} else {
				const uint32_t k = i - nW0 - nWh;
				o = ep.oWo + (4 * ((k / ep.W) & 3) + (k / ep.W) / 4) * ep.RSW + k % ep.W;  // out_row (mlp_fused.h)
			}
			ep.wimage[o] = h;
		}
	}
	if (g == 0) {
		__syncthreads();
		const float l = block_sum_fixed(ep.lpart, ep.n_wparts, lds);
		if (threadIdx.x == 0) *ep.d_loss = l;
	}
}

// The work plan by value (kernel arguments, read with scalar loads): the first thing every workgroup
// needs, so it must not cost a dependent global load at the head of the launch (r06). Plans larger
// than the tables keep reading the device copies.
constexpr uint32_t GRID_BWD_ARG_ITEMS = 32, GRID_BWD_ARG_LEVELS = 24;
struct GridBwdTables {
	uint32_t n_items, n_levels;  // entries valid below (0: read the device arrays)
	GridSlice items[GRID_BWD_ARG_ITEMS];
	LevelInfo levels[GRID_BWD_ARG_LEVELS];
};

template <uint32_t D, uint32_t F, HashType H, bool OPTS>
__global__ __launch_bounds__(GRID_BWD_THREADS) void k_grid_bwd_lds(
	int layout, uint32_t B, const float* __restrict__ pos, uint32_t pstride, const _Float16* __restrict__ dLdy, uint32_t dy_stride,
	const GridSlice* __restrict__ items, float* __restrict__ partial, uint32_t partial_stride,
	const LevelInfo* __restrict__ levels, uint32_t hash_grid, uint32_t interp_u, uint32_t pts_per_chunk, uint32_t n_items,
	uint32_t n_chunks, const GridBwdEpilogue ep, unsigned long long* dbg_times, const GridOpts o, const GridBwdTables tb) {
	extern __shared__ __attribute__((aligned(16))) int acc[];
	const unsigned long long t_start = dbg_times ? wall_clock64() : 0ull;
	__shared__ float red[GRID_BWD_THREADS / 64];
	if (blockIdx.x >= n_items * n_chunks) {
		grid_bwd_mlp_tail(ep, blockIdx.x - n_items * n_chunks, (float*)acc);
		if (dbg_times && threadIdx.x == 0) {
			dbg_times[8 * blockIdx.x] = t_start;
			for (int k = 1; k < 5; ++k) dbg_times[8 * blockIdx.x + k] = wall_clock64();
		}
		return;
	}
	// chunk-minor numbering: blocks are dealt round-robin over the 8 XCDs, so with 8 chunks every
	// item of chunk c lands on one XCD and the chunk's positions (re-read by all 26 items of
	// config_hash) stay in that XCD's L2
	const uint32_t item = blockIdx.x / n_chunks, chunk = blockIdx.x % n_chunks;
	GridSlice it;
	if (item < tb.n_items) {  // wave-uniform: scalar loads from the kernel arguments
		it.level = tb.items[item].level;
		it.begin = tb.items[item].begin;
		it.end = tb.items[item].end;
		it.f0 = tb.items[item].f0;
		it.nf = tb.items[item].nf;
	} else {
		it = items[item];
	}
	const uint32_t len = it.end - it.begin;
	const uint32_t nf = it.nf, f0 = it.f0;
	const Interp interp = (Interp)interp_u;
	const uint32_t i0 = chunk * pts_per_chunk;
	const uint32_t i1 = min(B, i0 + pts_per_chunk);

	// pre-pass: sum of |dL/dy| of this item's features over the chunk -> fixed-point scale. No entry
	// can receive more than that sum (the corner weights of a point sum to 1, hash collisions
	// included), so 2^e (sum + rounding) < 2^31 cannot overflow, and one outlier dL/dy costs the
	// other entries almost no resolution (a max-based bound would lose its whole ratio to the mean).
	// A non-finite dL/dy makes the item's gradient NaN (the reference's fp16 sums would carry it).
	float m = 0.0f;
	// D == 2, F <= 2 without grid options, and a chunk of at most GRID_BWD_PR points per thread (the
	// config_hash step: 32768-point chunks): the chunk's dL/dy bits are loaded once, all of them in
	// flight together, kept in registers for the accumulation, and the pre-pass is one load latency
	// instead of one per 8 points. The loads are issued first -- they need only the item -- so the
	// level table's load and the accumulators' zeroing run in their shadow (r05: at 2^15 points the
	// item load -> level load -> zeroing -> dL/dy load chain was ~5 us of a 13 us item)
	constexpr bool REGS_OK = D == 2 && F <= 2 && !OPTS;
	const uint32_t n_pts = i1 > i0 ? i1 - i0 : 0u;
	const bool use_regs = REGS_OK && n_pts <= GRID_BWD_THREADS * GRID_BWD_PR;
	uint32_t dyb[GRID_BWD_PR];
	float xs0[GRID_BWD_PU][D];  // the accumulation's first position batch, in flight across the scale reduction
	if constexpr (REGS_OK) {
		if (use_regs) {
#pragma unroll
			for (uint32_t p = 0; p < GRID_BWD_PR; ++p) {
				const uint32_t i = i0 + threadIdx.x + p * blockDim.x;
				dyb[p] = i < i1 ? load_dy_bits<F>(layout, dLdy, dy_stride, it.level, B, i) : 0u;
			}
			load_pos_batch<D>(pos, pstride, i0, i1, 0, xs0);
		}
	}
	LevelInfo li;
	if (it.level < tb.n_levels) {
		li.scale = tb.levels[it.level].scale;
		li.res = tb.levels[it.level].res;
		li.offset = tb.levels[it.level].offset;
		li.size = tb.levels[it.level].size;
	} else {
		li = levels[it.level];
	}
	// Replicas: a small level's accumulators fit the LDS several times; wave w adds into replica
	// w % R, which divides the same-address atomic serialisation on the coarse dense levels
	// (level 0: 256 entries hit by every point) by up to R. Integer sums: the replica merge below is
	// exact and order-independent.
	const uint32_t slots = len * nf;  // int32 slots of one replica (F = 2 packed pairs: 2 per entry)
	const uint32_t R = max(1u, min(16u, GRID_BWD_SLOTS / max(slots, 1u)));
	const uint32_t nz = R * slots;
	for (uint32_t j = 4 * threadIdx.x; j + 4 <= nz; j += 4 * blockDim.x) *(int4*)(acc + j) = int4{0, 0, 0, 0};  // ds_write_b128
	for (uint32_t j = nz / 4 * 4 + threadIdx.x; j < nz; j += blockDim.x) acc[j] = 0;
	if (dbg_times && threadIdx.x == 0) dbg_times[8 * blockIdx.x + 6] = wall_clock64();  // zeroing issued
	int* acc_w = acc + ((threadIdx.x >> 6) % R) * slots;
	if constexpr (REGS_OK) {
		if (use_regs) {
#pragma unroll
			for (uint32_t p = 0; p < GRID_BWD_PR; ++p) {
				float s = 0.0f;
#pragma unroll
				for (uint32_t f = 0; f < F; ++f) {
					const float v = dy_bits_feature(dyb[p], f);
					if (f - f0 < nf) s = __builtin_isfinite(v) ? fmaxf(s, fabsf(v)) : __builtin_inff();
				}
				m += s;
			}
		}
	}
	if (!use_regs) {
		for (uint32_t ib = i0 + threadIdx.x; ib < i1; ib += 8 * blockDim.x) {
			float dy[8][F];
#pragma unroll
			for (uint32_t u = 0; u < 8; ++u) {
				const uint32_t i = ib + u * blockDim.x;
				if (i < i1) load_dy<F>(layout, dLdy, dy_stride, it.level, B, i, dy[u]);
				else {
#pragma unroll
					for (uint32_t f = 0; f < F; ++f) dy[u][f] = 0.0f;
				}
			}
#pragma unroll
			for (uint32_t u = 0; u < 8; ++u) {
				float s = 0.0f;
#pragma unroll
				for (uint32_t f = 0; f < F; ++f)
					if (f - f0 < nf) s = __builtin_isfinite(dy[u][f]) ? fmaxf(s, fabsf(dy[u][f])) : __builtin_inff();
				m += s;
			}
		}
	}
	if (dbg_times && threadIdx.x == 0) dbg_times[8 * blockIdx.x + 5] = wall_clock64() + (m != m ? 1 : 0);  // dL/dy loads done
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) m += __shfl_xor(m, o);
	if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
	__syncthreads();
	m = red[0];
#pragma unroll
	for (uint32_t w = 1; w < GRID_BWD_THREADS / 64; ++w) m += red[w];
	const float P = (float)(i1 > i0 ? i1 - i0 : 1u);
	const bool finite = __builtin_isfinite(m);
	int e = 0;
	if (m > 0.0f && finite) {
		const float lim = (2147483647.0f - (float)(1u << D) * P) / (m * 1.01f);
		e = ilogbf(lim);  // floor(log2(lim))
		e = max(-126, min(e, 100));
	}
	const float scale = ldexpf(1.0f, e);
	if (dbg_times && threadIdx.x == 0) dbg_times[8 * blockIdx.x + 1] = wall_clock64();  // zeroing + pre-pass done

	// uniform per item: index kind and accumulation mode
	uint64_t full = 1;
	for (uint32_t d = 0; d < D; ++d) full = full * li.res > 0xffffffffull ? 0x100000000ull : full * li.res;
	const bool whole = it.begin == 0 && len == li.size;
	int kind = IDX_GENERIC;
	if (whole && full <= li.size) kind = IDX_DENSE;
	else if (whole && hash_grid && (li.size & (li.size - 1)) == 0) kind = IDX_HASH_POW2;
	else if (!whole && hash_grid && (li.size & (li.size - 1)) == 0 && full > li.size) kind = IDX_HASH_RANGE;
	const int mode = nf < F ? 1 : (F == 2 ? 0 : 2);
	if constexpr (REGS_OK) {
		if (use_regs) {
			if (kind == IDX_HASH_POW2)
				grid_bwd_mode_regs<D, F, H, IDX_HASH_POW2>(mode, dyb, xs0, B, pos, pstride, it.level, li, hash_grid != 0, interp, it.begin, len, f0, nf, i0, i1, scale, acc_w, o);
			else if (kind == IDX_HASH_RANGE)
				grid_bwd_mode_regs<D, F, H, IDX_HASH_RANGE>(mode, dyb, xs0, B, pos, pstride, it.level, li, hash_grid != 0, interp, it.begin, len, f0, nf, i0, i1, scale, acc_w, o);
			else if (kind == IDX_DENSE)
				grid_bwd_mode_regs<D, F, H, IDX_DENSE>(mode, dyb, xs0, B, pos, pstride, it.level, li, hash_grid != 0, interp, it.begin, len, f0, nf, i0, i1, scale, acc_w, o);
			else
				grid_bwd_mode_regs<D, F, H, IDX_GENERIC>(mode, dyb, xs0, B, pos, pstride, it.level, li, hash_grid != 0, interp, it.begin, len, f0, nf, i0, i1, scale, acc_w, o);
		}
	}
	if (!use_regs) {
	if (kind == IDX_HASH_POW2)
		grid_bwd_mode<D, F, H, IDX_HASH_POW2, OPTS>(mode, layout, B, pos, pstride, dLdy, dy_stride, it.level, li, hash_grid != 0, interp, it.begin, len, f0, nf, i0, i1, scale, acc_w, o);
	else if (kind == IDX_HASH_RANGE)
		grid_bwd_mode<D, F, H, IDX_HASH_RANGE, OPTS>(mode, layout, B, pos, pstride, dLdy, dy_stride, it.level, li, hash_grid != 0, interp, it.begin, len, f0, nf, i0, i1, scale, acc_w, o);
	else if (kind == IDX_DENSE)
		grid_bwd_mode<D, F, H, IDX_DENSE, OPTS>(mode, layout, B, pos, pstride, dLdy, dy_stride, it.level, li, hash_grid != 0, interp, it.begin, len, f0, nf, i0, i1, scale, acc_w, o);
	else
		grid_bwd_mode<D, F, H, IDX_GENERIC, OPTS>(mode, layout, B, pos, pstride, dLdy, dy_stride, it.level, li, hash_grid != 0, interp, it.begin, len, f0, nf, i0, i1, scale, acc_w, o);
	}
	__syncthreads();
	if (dbg_times && threadIdx.x == 0) dbg_times[8 * blockIdx.x + 2] = wall_clock64();  // accumulation done
	if (R > 1) {  // merge the replicas into replica 0
		if (mode == 0) {
			long long* a64 = (long long*)acc;
			for (uint32_t j = threadIdx.x; j < len; j += blockDim.x) {
				long long t = a64[j];
				for (uint32_t r = 1; r < R; ++r) t += a64[(size_t)r * len + j];
				a64[j] = t;
			}
		} else {
			for (uint32_t j = threadIdx.x; j < slots; j += blockDim.x) {
				int t = acc[j];
				for (uint32_t r = 1; r < R; ++r) t += acc[(size_t)r * slots + j];
				acc[j] = t;
			}
		}
		__syncthreads();
	}
	if (dbg_times && threadIdx.x == 0) dbg_times[8 * blockIdx.x + 3] = wall_clock64();  // replica merge done
	// write the chunk slab (GridSlabMap layout: this item's accumulators are one contiguous range)
	const float inv = finite ? ldexpf(1.0f, -e) : __builtin_nanf("");
	float* dst = partial + (size_t)chunk * partial_stride + (size_t)li.offset * F + (size_t)f0 * li.size + (size_t)it.begin * nf;
	if (mode == 0) {  // decode the packed int32 pairs, two entries per thread (16-byte stores)
		const long long* a64 = (const long long*)acc;
		auto dec = [&](long long t) {
			const int lo = (int)(uint32_t)(unsigned long long)t;
			const int hi = (int)((t - (long long)lo) >> 32);
			return make_float2((float)lo * inv, (float)hi * inv);
		};
		const bool al = (((uintptr_t)dst) & 15) == 0;
		for (uint32_t j = 2 * threadIdx.x; j < len; j += 2 * blockDim.x) {
			const float2 a = dec(a64[j]);
			if (al && j + 1 < len) {
				const float2 b = dec(a64[j + 1]);
				*(f4*)(dst + 2 * j) = f4{a.x, a.y, b.x, b.y};
			} else {
				*(float2*)(dst + 2 * j) = a;
				if (j + 1 < len) *(float2*)(dst + 2 * j + 2) = dec(a64[j + 1]);
			}
		}
	} else {
		const uint32_t n = len * nf;
		const bool al = (((uintptr_t)dst) & 15) == 0;
		for (uint32_t j = 4 * threadIdx.x; j < n; j += 4 * blockDim.x) {
			if (al && j + 4 <= n) {
				const int4 v = *(const int4*)(acc + j);
				*(f4*)(dst + j) = f4{(float)v.x * inv, (float)v.y * inv, (float)v.z * inv, (float)v.w * inv};
			} else {
				for (uint32_t k = j; k < n && k < j + 4; ++k) dst[k] = (float)acc[k] * inv;
			}
		}
	}
	if (dbg_times && threadIdx.x == 0) {
		dbg_times[8 * blockIdx.x] = t_start;
		dbg_times[8 * blockIdx.x + 4] = wall_clock64();
	}
}

struct GridBwdLaunch {
	uint32_t n_items, n_chunks;
	GridBwdEpilogue ep;
	unsigned long long* dbg_times;
	GridOpts opts;
	GridBwdTables tb;
};

template <uint32_t D, uint32_t F, HashType H>
static void grid_bwd_t(hipStream_t st, int layout, uint32_t dys, dim3 g, size_t lds, uint32_t B, const float* pos, uint32_t ps,
                       const _Float16* dy, const GridSlice* sl, float* part, uint32_t pstr, const LevelInfo* lv,
                       uint32_t hg, uint32_t in, uint32_t ppc, const GridBwdLaunch& gl) {
	// the options (max_level, stochastic) are a separate instantiation: the default kernel stays lean
	static uint64_t done0 = 0, done1 = 0;
	set_dyn_lds((const void*)k_grid_bwd_lds<D, F, H, false>, (int)GRID_BWD_LDS_BYTES, done0);
	set_dyn_lds((const void*)k_grid_bwd_lds<D, F, H, true>, (int)GRID_BWD_LDS_BYTES, done1);
	if (gl.opts.active)
		hipLaunchKernelGGL((k_grid_bwd_lds<D, F, H, true>), g, dim3(GRID_BWD_THREADS), lds, st, layout, B, pos, ps, dy, dys, sl, part, pstr, lv, hg, in,
		                   ppc, gl.n_items, gl.n_chunks, gl.ep, gl.dbg_times, gl.opts, gl.tb);
	else
		hipLaunchKernelGGL((k_grid_bwd_lds<D, F, H, false>), g, dim3(GRID_BWD_THREADS), lds, st, layout, B, pos, ps, dy, dys, sl, part, pstr, lv, hg, in,
		                   ppc, gl.n_items, gl.n_chunks, gl.ep, gl.dbg_times, gl.opts, gl.tb);
}

template <uint32_t D, uint32_t F>
static void grid_bwd_h(hipStream_t st, HashType h, int pairs, uint32_t dys, dim3 g, size_t lds, uint32_t B, const float* pos, uint32_t ps,
                       const _Float16* dy, const GridSlice* sl, float* part, uint32_t pstr, const LevelInfo* lv,
                       uint32_t hg, uint32_t in, uint32_t ppc, const GridBwdLaunch& gl) {
	switch (h) {
		case HashType::Prime: grid_bwd_t<D, F, HashType::Prime>(st, pairs, dys, g, lds, B, pos, ps, dy, sl, part, pstr, lv, hg, in, ppc, gl); break;
		case HashType::ReversedPrime: grid_bwd_t<D, F, HashType::ReversedPrime>(st, pairs, dys, g, lds, B, pos, ps, dy, sl, part, pstr, lv, hg, in, ppc, gl); break;
		default: grid_bwd_t<D, F, HashType::CoherentPrime>(st, pairs, dys, g, lds, B, pos, ps, dy, sl, part, pstr, lv, hg, in, ppc, gl); break;
	}
}

template <uint32_t D>
void grid_bwd_f(hipStream_t st, uint32_t F, HashType h, int pairs, uint32_t dys, dim3 g, size_t lds, uint32_t B, const float* pos,
                       uint32_t ps, const _Float16* dy, const GridSlice* sl, float* part, uint32_t pstr, const LevelInfo* lv,
                       uint32_t hg, uint32_t in, uint32_t ppc, const GridBwdLaunch& gl) {
	switch (F) {
		case 1: grid_bwd_h<D, 1>(st, h, pairs, dys, g, lds, B, pos, ps, dy, sl, part, pstr, lv, hg, in, ppc, gl); break;
		case 2: grid_bwd_h<D, 2>(st, h, pairs, dys, g, lds, B, pos, ps, dy, sl, part, pstr, lv, hg, in, ppc, gl); break;
		case 4: grid_bwd_h<D, 4>(st, h, pairs, dys, g, lds, B, pos, ps, dy, sl, part, pstr, lv, hg, in, ppc, gl); break;
		case 8: grid_bwd_h<D, 8>(st, h, pairs, dys, g, lds, B, pos, ps, dy, sl, part, pstr, lv, hg, in, ppc, gl); break;
		default: throw std::runtime_error("GridEncoding: n_features_per_level must be 1, 2, 4 or 8");
	}
}

}  // namespace tcnn_amd
