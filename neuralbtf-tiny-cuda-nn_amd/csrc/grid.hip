// grid.hip -- multiresolution grid encoding kernels for gfx950:
//   k_grid_fwd      standalone grid forward (reference grid.h:48-212)
//   k_grid_bwd_lds  grid backward, LDS-privatised per (level, entries x features, point chunk)
//                   (reference grid.h:214-320; int32 fixed-point sums instead of fp16 atomics)
#include "kernels.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "adam_device.h"
#include "grid_device.h"

namespace tcnn_amd {
// =============================================================================================
// grid forward (standalone)
// =============================================================================================

template <uint32_t F>
struct HVec { _Float16 v[F]; };

template <uint32_t D, uint32_t F, HashType H>
__global__ __launch_bounds__(256) void k_grid_fwd(uint32_t B, const float* __restrict__ pos, uint32_t pstride,
                                                  const _Float16* __restrict__ table, _Float16* __restrict__ out,
                                                  uint32_t soa, uint32_t out_stride, const LevelInfo* __restrict__ levels,
                                                  uint32_t hash_grid, uint32_t interp_u, const GridOpts o, uint32_t L) {
	// SoA output: lanes = consecutive points of one level (blockIdx.y); AoS rows: lanes = the levels of
	// consecutive points, so one store instruction writes whole rows
	uint32_t i, level;
	if (soa) {
		i = blockIdx.x * blockDim.x + threadIdx.x;
		level = blockIdx.y;
	} else {
		const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
		i = t / L;
		level = t % L;
	}
	if (i >= B) return;
	const LevelInfo li = levels[level];
	const Interp interp = (Interp)interp_u;
	float p[D];
	uint32_t pg[D];
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) pos_fract(pos[(size_t)i * pstride + d], li.scale, interp, p[d], pg[d]);
	_Float16 r[F];
#pragma unroll
	for (uint32_t f = 0; f < F; ++f) r[f] = (_Float16)0.0f;
	const HVec<F>* tv = (const HVec<F>*)table;
	if (o.active && (float)level >= grid_max_level(o, i, F) + 1e-3f) {
		// masked level: output 0 (grid.h:75-91)
	} else if (interp == Interp::Nearest) {
		const HVec<F> v = tv[li.offset + grid_index<D, H>(hash_grid != 0, li.size, li.res, pg)];
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) r[f] = v.v[f];
	} else {
		constexpr uint32_t NC = 1u << D;
		HVec<F> v[NC];
		_Float16 w16[NC];
#pragma unroll
		for (uint32_t c = 0; c < NC; ++c) {
			float w = 1.0f;
			uint32_t local[D];
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) {
				if ((c & (1u << d)) == 0) { w *= 1.0f - p[d]; local[d] = pg[d]; }
				else { w *= p[d]; local[d] = pg[d] + 1; }
			}
			w16[c] = (_Float16)w;
			v[c] = tv[li.offset + grid_index<D, H>(hash_grid != 0, li.size, li.res, local)];
		}
		// packed fp16 FMA (v_pk_fma_f16: one rounding, = CUDA __hfma2 of grid.h:162); the scalar
		// _Float16 fma is lowered through fp32 and would double-round.
#pragma unroll
		for (uint32_t c = 0; c < NC; ++c) {
			const h2 wv = {w16[c], w16[c]};
#pragma unroll
			for (uint32_t f = 0; f < F; f += 2) {
				h2 vv, rr;
				vv[0] = v[c].v[f]; vv[1] = (f + 1 < F) ? v[c].v[f + 1] : (_Float16)0.0f;
				rr[0] = r[f]; rr[1] = (f + 1 < F) ? r[f + 1] : (_Float16)0.0f;
				rr = pk_fma_f16(wv, vv, rr);
				r[f] = rr[0];
				if (f + 1 < F) r[f + 1] = rr[1];
			}
		}
	}
	if (soa) {
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) out[(size_t)(level * F + f) * B + i] = r[f];
	} else {
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) out[(size_t)i * out_stride + level * F + f] = r[f];
	}
}

template <uint32_t D, uint32_t F>
static void grid_fwd_h(hipStream_t st, HashType h, dim3 g, uint32_t B, const float* pos, uint32_t ps, const _Float16* t,
                       _Float16* o, uint32_t soa, uint32_t os, const LevelInfo* lv, uint32_t hg, uint32_t in, const GridOpts& go) {
	const uint32_t L = soa ? g.y : go.n_levels;
	switch (h) {
		case HashType::Prime: hipLaunchKernelGGL((k_grid_fwd<D, F, HashType::Prime>), g, dim3(256), 0, st, B, pos, ps, t, o, soa, os, lv, hg, in, go, L); break;
		case HashType::ReversedPrime: hipLaunchKernelGGL((k_grid_fwd<D, F, HashType::ReversedPrime>), g, dim3(256), 0, st, B, pos, ps, t, o, soa, os, lv, hg, in, go, L); break;
		default: hipLaunchKernelGGL((k_grid_fwd<D, F, HashType::CoherentPrime>), g, dim3(256), 0, st, B, pos, ps, t, o, soa, os, lv, hg, in, go, L); break;
	}
}

template <uint32_t D>
static void grid_fwd_f(hipStream_t st, uint32_t F, HashType h, dim3 g, uint32_t B, const float* pos, uint32_t ps,
                       const _Float16* t, _Float16* o, uint32_t soa, uint32_t os, const LevelInfo* lv, uint32_t hg, uint32_t in,
                       const GridOpts& go) {
	switch (F) {
		case 1: grid_fwd_h<D, 1>(st, h, g, B, pos, ps, t, o, soa, os, lv, hg, in, go); break;
		case 2: grid_fwd_h<D, 2>(st, h, g, B, pos, ps, t, o, soa, os, lv, hg, in, go); break;
		case 4: grid_fwd_h<D, 4>(st, h, g, B, pos, ps, t, o, soa, os, lv, hg, in, go); break;
		case 8: grid_fwd_h<D, 8>(st, h, g, B, pos, ps, t, o, soa, os, lv, hg, in, go); break;
		default: throw std::runtime_error("GridEncoding: n_features_per_level must be 1, 2, 4 or 8");
	}
}

void launch_grid_fwd(hipStream_t st, uint32_t D, uint32_t F, HashType h, uint32_t B, uint32_t L,
                     const float* pos, uint32_t pos_stride, const void* table16, void* out16, bool soa,
                     uint32_t out_stride, const LevelInfo* levels, bool hash_grid, Interp interp, const GridOpts& go) {
	if (B == 0) return;
	const dim3 g = soa ? dim3(div_round_up(B, 256), L) : dim3(div_round_up(B * L, 256), 1);
	GridOpts gol = go;
	gol.n_levels = L;  // carries L to the AoS mapping
	const _Float16* t = (const _Float16*)table16;
	_Float16* o = (_Float16*)out16;
	switch (D) {
		case 2: grid_fwd_f<2>(st, F, h, g, B, pos, pos_stride, t, o, soa, out_stride, levels, hash_grid, (uint32_t)interp, gol); break;
		case 3: grid_fwd_f<3>(st, F, h, g, B, pos, pos_stride, t, o, soa, out_stride, levels, hash_grid, (uint32_t)interp, gol); break;
		case 4: grid_fwd_f<4>(st, F, h, g, B, pos, pos_stride, t, o, soa, out_stride, levels, hash_grid, (uint32_t)interp, gol); break;
		default: throw std::runtime_error("GridEncoding: number of input dims must be 2, 3 or 4");
	}
	TCNN_HIP_CHECK(hipGetLastError());
}

// =============================================================================================
// grid backward: LDS-privatised slices
// =============================================================================================

// LDS accumulators are int32 fixed point with a per-(work item, chunk) power-of-two scale.
// gfx950 executes LDS float atomics (ds_add_f32 / ds_pk_add_f16) at ~195 cycles per wave-instruction
// per CU but ds_add_u32 at ~8 (tools/lds_atomic_bench.hip), and integer sums are order-independent,
// so the gradient is bit-reproducible (the reference's fp16 atomics, grid.h:252-255, are not).
// Range: the bilinear weights of one point sum to 1, so no table entry can receive more than
// P * max|dL/dy| from a chunk of P points (hash collisions included); the scale 2^e is the largest
// power of two that keeps that bound plus the rounding of every add below 2^31. At B = 2^18 split
// into ~10 chunks that leaves ~2^-16 * max|dL/dy| per add -- finer than the reference's fp16 sums.
// 32-bit accumulators let a whole 32768-entry hashed level (one feature) or a whole dense level
// (all features) sit in 128 KiB of LDS: every corner update lands, no lane is masked off, and each
// point is visited by 26 work items (config_hash) instead of 47 entry slices.
constexpr uint32_t GRID_BWD_THREADS = 1024;
constexpr uint32_t GRID_BWD_LDS_BYTES = 128 * 1024;
constexpr uint32_t GRID_BWD_SLOTS = GRID_BWD_LDS_BYTES / 4;

uint32_t grid_bwd_slot_budget() { return GRID_BWD_SLOTS; }

__device__ __forceinline__ void lds_add_i32(int* acc, float v) {
	__hip_atomic_fetch_add(acc, __float2int_rn(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <uint32_t F>
__device__ __forceinline__ void load_dy(int layout, const _Float16* __restrict__ dLdy, uint32_t dy_stride, uint32_t level, uint32_t B,
                                        uint32_t i, float* dy) {
	if (layout == 0) {  // level-major feature pairs [l][i][F]
		const HVec<F> v = ((const HVec<F>*)dLdy)[(size_t)level * B + i];
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) dy[f] = (float)v.v[f];
	} else if (layout == 1) {  // SoA [(l*F+f)*B + i] (reference RM layout)
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) dy[f] = (float)dLdy[(size_t)(level * F + f) * B + i];
	} else {  // AoS [i*stride + l*F + f] (reference CM layout)
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) dy[f] = (float)dLdy[(size_t)i * dy_stride + level * F + f];
	}
}

// Index kinds of a level, uniform per work item (reference grid_index, common_device.h:690-707):
//   HASH_POW2  hashed level of power-of-two size: index = hash & (size - 1)
//   DENSE      res^D <= size: index = sum g_d res^d, < 2 size, so `% size` is one conditional subtract
//   GENERIC    anything else (tiled grids, non-power-of-two hashed sizes): grid_index()
enum : int { IDX_HASH_POW2 = 0, IDX_DENSE = 1, IDX_GENERIC = 2 };

template <uint32_t D, HashType H, int KIND>
__device__ __forceinline__ uint32_t level_index(bool hash_grid, uint32_t size, uint32_t res, const uint32_t* g) {
	if constexpr (KIND == IDX_HASH_POW2) {
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
		return idx >= size ? idx - size : idx;
	} else {
		return grid_index<D, H>(hash_grid, size, res, g);
	}
}

// MODE: 0 = F == 2, both features as one packed int64 (two int32 halves) per entry -> one
// ds_add_u64 per corner; 1 = one feature (f0) per entry, ds_add_u32; 2 = all F features, ds_add_u32.
template <uint32_t D, uint32_t F, HashType H, int KIND, int MODE, bool OPTS>
__device__ __forceinline__ void grid_bwd_points(int layout, uint32_t B, const float* __restrict__ pos, uint32_t pstride,
                                                const _Float16* __restrict__ dLdy, uint32_t dy_stride, uint32_t level,
                                                const LevelInfo& li, bool hash_grid, Interp interp, uint32_t begin,
                                                uint32_t len, uint32_t f0, uint32_t i0, uint32_t i1, float scale, int* acc,
                                                const GridOpts& o) {
	constexpr uint32_t NF = MODE == 1 ? 1 : F;
	constexpr uint32_t U = 8;  // points in flight per thread
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
			if constexpr (MODE == 1) {
				float s = v[0];
#pragma unroll
				for (uint32_t f = 1; f < F; ++f) s = f == f0 ? v[f] : s;
				dy[u][0] = s * scale;
			} else {
#pragma unroll
				for (uint32_t f = 0; f < F; ++f) dy[u][f] = v[f] * scale;
			}
		}
#pragma unroll
		for (uint32_t u = 0; u < U; ++u) {
			if (base + u * blockDim.x >= i1) break;
			float p[D];
			uint32_t pg[D];
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) pos_fract(xs[u][d], li.scale, interp, p[d], pg[d]);
			const bool nearest = interp == Interp::Nearest;
			// stochastic interpolation (grid.h:284-298): one corner, chosen per (point, level), weight 1
			const bool single = nearest || (OPTS && o.stochastic);
			uint32_t cbits = 0;
			if (single && !nearest) {
				const float smp = random_val_1337(base + u * blockDim.x + level * B);
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
				const float wh = single ? 1.0f : (float)(_Float16)w;
				const uint32_t rel = level_index<D, H, KIND>(hash_grid, li.size, li.res, local) - begin;
				if constexpr (KIND == IDX_GENERIC) {  // entry slices may not cover the level
					if (rel >= len) continue;
				}
				if constexpr (MODE == 0) {
					const int a = __float2int_rn(wh * dy[u][0]);
					const int b = __float2int_rn(wh * dy[u][1]);
					const unsigned long long pk = (unsigned long long)(((long long)b << 32) + (long long)a);
					__hip_atomic_fetch_add((unsigned long long*)acc + rel, pk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
				} else {
#pragma unroll
					for (uint32_t f = 0; f < NF; ++f) lds_add_i32(&acc[rel * NF + f], wh * dy[u][f]);
				}
			}
		}
	}
}

template <uint32_t D, uint32_t F, HashType H, int KIND, bool OPTS>
__device__ __forceinline__ void grid_bwd_mode(int mode, int layout, uint32_t B, const float* pos, uint32_t pstride,
                                              const _Float16* dLdy, uint32_t dy_stride, uint32_t level, const LevelInfo& li,
                                              bool hash_grid, Interp interp, uint32_t begin, uint32_t len, uint32_t f0,
                                              uint32_t i0, uint32_t i1, float scale, int* acc, const GridOpts& o) {
	if constexpr (F == 2) {
		if (mode == 0) { grid_bwd_points<D, F, H, KIND, 0, OPTS>(layout, B, pos, pstride, dLdy, dy_stride, level, li, hash_grid, interp, begin, len, f0, i0, i1, scale, acc, o); return; }
	} else if constexpr (F > 2) {
		if (mode == 2) { grid_bwd_points<D, F, H, KIND, 2, OPTS>(layout, B, pos, pstride, dLdy, dy_stride, level, li, hash_grid, interp, begin, len, f0, i0, i1, scale, acc, o); return; }
	}
	grid_bwd_points<D, F, H, KIND, 1, OPTS>(layout, B, pos, pstride, dLdy, dy_stride, level, li, hash_grid, interp, begin, len, f0, i0, i1, scale, acc, o);
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
				o = ep.oWo + (k / ep.W) * ep.RSW + k % ep.W;
			}
			ep.wimage[o] = h;
		}
	}
	if (g == 0) {
		__syncthreads();
		const float l = block_sum_fixed(ep.lpart, ep.n_wparts, lds);
		if (threadIdx.x == 0) {
			*ep.d_loss = l;
			if (ep.apply_adam && ep.factor_out) *ep.factor_out = adam_bias_factor(ep.adam_mlp, ep.factor_step);
		}
	}
}

template <uint32_t D, uint32_t F, HashType H, bool OPTS>
__global__ __launch_bounds__(GRID_BWD_THREADS) void k_grid_bwd_lds(
	int layout, uint32_t B, const float* __restrict__ pos, uint32_t pstride, const _Float16* __restrict__ dLdy, uint32_t dy_stride,
	const GridSlice* __restrict__ items, float* __restrict__ partial, uint32_t partial_stride,
	const LevelInfo* __restrict__ levels, uint32_t hash_grid, uint32_t interp_u, uint32_t pts_per_chunk, uint32_t n_items,
	uint32_t n_chunks, const GridBwdEpilogue ep, unsigned long long* dbg_times, const GridOpts o) {
	extern __shared__ __attribute__((aligned(16))) int acc[];
	const unsigned long long t_start = dbg_times ? wall_clock64() : 0ull;
	__shared__ float red[GRID_BWD_THREADS / 64];
	if (blockIdx.x >= n_items * n_chunks) {
		grid_bwd_mlp_tail(ep, blockIdx.x - n_items * n_chunks, (float*)acc);
		if (dbg_times && threadIdx.x == 0) {
			dbg_times[2 * blockIdx.x] = t_start;
			dbg_times[2 * blockIdx.x + 1] = wall_clock64();
		}
		return;
	}
	const uint32_t item = blockIdx.x % n_items, chunk = blockIdx.x / n_items;
	const GridSlice it = items[item];
	const LevelInfo li = levels[it.level];
	const uint32_t len = it.end - it.begin;
	const uint32_t nf = it.nf, f0 = it.f0;
	const Interp interp = (Interp)interp_u;
	// Replicas: a small level's accumulators fit the LDS several times; wave w adds into replica
	// w % R, which divides the same-address atomic serialisation on the coarse dense levels
	// (level 0: 256 entries hit by every point) by up to R. Integer sums: the replica merge below is
	// exact and order-independent.
	const uint32_t slots = len * nf;  // int32 slots of one replica (F = 2 packed pairs: 2 per entry)
	const uint32_t R = max(1u, min(16u, GRID_BWD_SLOTS / max(slots, 1u)));
	for (uint32_t j = threadIdx.x; j < R * slots; j += blockDim.x) acc[j] = 0;
	int* acc_w = acc + ((threadIdx.x >> 6) % R) * slots;
	const uint32_t i0 = chunk * pts_per_chunk;
	const uint32_t i1 = min(B, i0 + pts_per_chunk);

	// pre-pass: max |dL/dy| of this item's features over the chunk -> fixed-point scale
	// (8 independent loads in flight per thread)
	float m = 0.0f;
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
		for (uint32_t u = 0; u < 8; ++u)
#pragma unroll
			for (uint32_t f = 0; f < F; ++f)
				if (f - f0 < nf) m = fmaxf(m, fabsf(dy[u][f]));
	}
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
	if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
	__syncthreads();
	m = red[0];
#pragma unroll
	for (uint32_t w = 1; w < GRID_BWD_THREADS / 64; ++w) m = fmaxf(m, red[w]);
	const float P = (float)(i1 > i0 ? i1 - i0 : 1u);
	int e = 0;
	if (m > 0.0f && m <= 65504.0f) {
		const float lim = (2147483647.0f - 8.0f * P) / (P * m * 1.001f);
		e = ilogbf(lim);  // floor(log2(lim))
		e = max(-126, min(e, 100));
	}
	const float scale = ldexpf(1.0f, e);

	// uniform per item: index kind and accumulation mode
	uint64_t full = 1;
	for (uint32_t d = 0; d < D; ++d) full = full * li.res > 0xffffffffull ? 0x100000000ull : full * li.res;
	const bool whole = it.begin == 0 && len == li.size;
	int kind = IDX_GENERIC;
	if (whole && full <= li.size) kind = IDX_DENSE;
	else if (whole && hash_grid && (li.size & (li.size - 1)) == 0) kind = IDX_HASH_POW2;
	const int mode = nf == 1 ? 1 : (F == 2 ? 0 : 2);
	if (kind == IDX_HASH_POW2)
		grid_bwd_mode<D, F, H, IDX_HASH_POW2, OPTS>(mode, layout, B, pos, pstride, dLdy, dy_stride, it.level, li, hash_grid != 0, interp, it.begin, len, f0, i0, i1, scale, acc_w, o);
	else if (kind == IDX_DENSE)
		grid_bwd_mode<D, F, H, IDX_DENSE, OPTS>(mode, layout, B, pos, pstride, dLdy, dy_stride, it.level, li, hash_grid != 0, interp, it.begin, len, f0, i0, i1, scale, acc_w, o);
	else
		grid_bwd_mode<D, F, H, IDX_GENERIC, OPTS>(mode, layout, B, pos, pstride, dLdy, dy_stride, it.level, li, hash_grid != 0, interp, it.begin, len, f0, i0, i1, scale, acc_w, o);
	__syncthreads();
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
	// write the chunk slab (GridSlabMap layout: this item's accumulators are one contiguous range)
	const float inv = ldexpf(1.0f, -e);
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
		dbg_times[2 * blockIdx.x] = t_start;
		dbg_times[2 * blockIdx.x + 1] = wall_clock64();
	}
}

// dL/dx through the grid (reference kernel_grid's dy_dx branch, grid.h:171-211, and
// kernel_grid_backward_input, grid.h:322-349), fused: dy_dx is recomputed per point from the table
// instead of being stored by the forward ([L*F][B][D] fp32 = 256 B/sample of HBM traffic saved).
// Same operation order and FMA contraction points as the reference (see the oracle).
template <uint32_t D, uint32_t F, HashType H>
__global__ __launch_bounds__(256) void k_grid_bwd_input(uint32_t B, uint32_t L, const float* __restrict__ pos, uint32_t pstride,
                                                        const _Float16* __restrict__ table, const _Float16* __restrict__ dLdy,
                                                        int layout, uint32_t dy_stride, float* __restrict__ dx, uint32_t dx_stride,
                                                        const LevelInfo* __restrict__ levels, uint32_t hash_grid, uint32_t interp_u,
                                                        const GridOpts o) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= B) return;
	const Interp interp = (Interp)interp_u;
	const float ml = o.active ? grid_max_level(o, i, F) + 1e-3f : 3.0e38f;
	float x[D], res[D];
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) {
		x[d] = pos[(size_t)i * pstride + d];
		res[d] = 0.0f;
	}
	for (uint32_t l = 0; l < L; ++l) {
		if ((float)l >= ml) continue;  // masked: dy_dx = 0 (grid.h:75-91)
		const LevelInfo li = levels[l];
		float p[D], pd[D];
		uint32_t pg[D];
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) {
			float v = __builtin_fmaf(li.scale, x[d], 0.5f);
			const float t = floorf(v);
			pg[d] = (uint32_t)(int)t;
			v -= t;
			if (interp == Interp::Smoothstep) {
				pd[d] = 6.0f * v * (1.0f - v);
				v = v * v * __builtin_fmaf(-2.0f, v, 3.0f);
			} else {
				pd[d] = 1.0f;
			}
			p[d] = v;
		}
		float grads[F][D];
#pragma unroll
		for (uint32_t f = 0; f < F; ++f)
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) grads[f][d] = 0.0f;
		if (interp != Interp::Nearest) {
#pragma unroll
			for (uint32_t gd = 0; gd < D; ++gd) {
#pragma unroll
				for (uint32_t idx = 0; idx < (1u << (D - 1)); ++idx) {
					float w = li.scale;
					uint32_t local[D];
#pragma unroll
					for (uint32_t nd = 0; nd < D - 1; ++nd) {
						const uint32_t dim = nd >= gd ? nd + 1 : nd;
						if ((idx & (1u << nd)) == 0) { w *= 1.0f - p[dim]; local[dim] = pg[dim]; }
						else { w *= p[dim]; local[dim] = pg[dim] + 1; }
					}
					local[gd] = pg[gd];
					const size_t il = (size_t)(li.offset + grid_index<D, H>(hash_grid != 0, li.size, li.res, local)) * F;
					local[gd] = pg[gd] + 1;
					const size_t ir = (size_t)(li.offset + grid_index<D, H>(hash_grid != 0, li.size, li.res, local)) * F;
#pragma unroll
					for (uint32_t f = 0; f < F; ++f) {
						const float diff = (float)table[ir + f] - (float)table[il + f];
						grads[f][gd] = __builtin_fmaf(w * diff, pd[gd], grads[f][gd]);
					}
				}
			}
		}
		float dy[F];
		load_dy<F>(layout, dLdy, dy_stride, l, B, i, dy);
#pragma unroll
		for (uint32_t f = 0; f < F; ++f)
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) res[d] = __builtin_fmaf(dy[f], grads[f][d], res[d]);
	}
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) dx[(size_t)i * dx_stride + d] = res[d];
}

template <uint32_t D, uint32_t F>
static void grid_bwd_input_h(hipStream_t st, HashType h, dim3 g, uint32_t B, uint32_t L, const float* pos, uint32_t ps, const _Float16* t,
                             const _Float16* dy, int layout, uint32_t dys, float* dx, uint32_t dxs, const LevelInfo* lv, uint32_t hg,
                             uint32_t in, const GridOpts& go) {
	switch (h) {
		case HashType::Prime: hipLaunchKernelGGL((k_grid_bwd_input<D, F, HashType::Prime>), g, dim3(256), 0, st, B, L, pos, ps, t, dy, layout, dys, dx, dxs, lv, hg, in, go); break;
		case HashType::ReversedPrime: hipLaunchKernelGGL((k_grid_bwd_input<D, F, HashType::ReversedPrime>), g, dim3(256), 0, st, B, L, pos, ps, t, dy, layout, dys, dx, dxs, lv, hg, in, go); break;
		default: hipLaunchKernelGGL((k_grid_bwd_input<D, F, HashType::CoherentPrime>), g, dim3(256), 0, st, B, L, pos, ps, t, dy, layout, dys, dx, dxs, lv, hg, in, go); break;
	}
}

template <uint32_t D>
static void grid_bwd_input_f(hipStream_t st, uint32_t F, HashType h, dim3 g, uint32_t B, uint32_t L, const float* pos, uint32_t ps,
                             const _Float16* t, const _Float16* dy, int layout, uint32_t dys, float* dx, uint32_t dxs,
                             const LevelInfo* lv, uint32_t hg, uint32_t in, const GridOpts& go) {
	switch (F) {
		case 1: grid_bwd_input_h<D, 1>(st, h, g, B, L, pos, ps, t, dy, layout, dys, dx, dxs, lv, hg, in, go); break;
		case 2: grid_bwd_input_h<D, 2>(st, h, g, B, L, pos, ps, t, dy, layout, dys, dx, dxs, lv, hg, in, go); break;
		case 4: grid_bwd_input_h<D, 4>(st, h, g, B, L, pos, ps, t, dy, layout, dys, dx, dxs, lv, hg, in, go); break;
		case 8: grid_bwd_input_h<D, 8>(st, h, g, B, L, pos, ps, t, dy, layout, dys, dx, dxs, lv, hg, in, go); break;
		default: throw std::runtime_error("GridEncoding: n_features_per_level must be 1, 2, 4 or 8");
	}
}

void launch_grid_bwd_input(hipStream_t st, uint32_t D, uint32_t F, HashType h, uint32_t B, uint32_t L, const float* pos,
                           uint32_t pos_stride, const void* table16, const void* dLdy16, int dy_layout, uint32_t dy_stride, float* dx,
                           uint32_t dx_stride, const LevelInfo* levels, bool hash_grid, Interp interp, const GridOpts& go) {
	if (B == 0) return;
	const dim3 g(div_round_up(B, 256));
	const _Float16* t = (const _Float16*)table16;
	const _Float16* dy = (const _Float16*)dLdy16;
	switch (D) {
		case 2: grid_bwd_input_f<2>(st, F, h, g, B, L, pos, pos_stride, t, dy, dy_layout, dy_stride, dx, dx_stride, levels, hash_grid, (uint32_t)interp, go); break;
		case 3: grid_bwd_input_f<3>(st, F, h, g, B, L, pos, pos_stride, t, dy, dy_layout, dy_stride, dx, dx_stride, levels, hash_grid, (uint32_t)interp, go); break;
		case 4: grid_bwd_input_f<4>(st, F, h, g, B, L, pos, pos_stride, t, dy, dy_layout, dy_stride, dx, dx_stride, levels, hash_grid, (uint32_t)interp, go); break;
		default: throw std::runtime_error("GridEncoding: number of input dims must be 2, 3 or 4");
	}
	TCNN_HIP_CHECK(hipGetLastError());
}


// ---------------------------------------------------------------------------------------------
// Second-order grid gradients: backward of backward_input (reference grid.h:351-627, host
// :902-1026). One thread per point walks all levels; per corner c of a level it forms
//   A_c      = sum_e g_e s pd_e sign_e(c) prod_{d!=e} w_d(c)          (d/dx of the corner weight . g)
//   K_e(c)   = s^2 [pd2_e g_e sign_e(c) prod_{d!=e} w_d + sum_{o!=e} pd_e pd_o g_o sign_e sign_o prod_{d!=e,o} w_d]
// so that dL/dgrid[c] += A_c dL/dy, dL/d(dL/dy) = sum_c A_c T[c], dL/dx_e = sum_c K_e(c) (T[c] . dL/dy)
// (g = dL/d(dL/dx); the reference's per-edge loops regrouped per corner; fp32 throughout, grid
// gradient by fp32 atomics). dLdy AoS fp16 [B][dy_stride]; dLddLdy AoS fp16 [B][ddy_stride] with
// the padding columns zeroed; dx fp32 [B][D] overwritten.
// ---------------------------------------------------------------------------------------------
template <uint32_t D, uint32_t F, HashType H>
__global__ __launch_bounds__(256) void k_grid_bwd_bwd(uint32_t B, uint32_t L, const float* __restrict__ pos, uint32_t pstride,
                                                      const _Float16* __restrict__ table, const float* __restrict__ gxx,
                                                      const _Float16* __restrict__ dLdy, uint32_t dy_stride, float* __restrict__ grad,
                                                      _Float16* __restrict__ dLddLdy, uint32_t ddy_stride, float* __restrict__ dx,
                                                      const LevelInfo* __restrict__ levels, uint32_t hash_grid, uint32_t interp_u,
                                                      const GridOpts o) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= B) return;
	const Interp interp = (Interp)interp_u;
	// forward-side mask (dy_dx = 0, grid.h:75) uses >=, the second-order kernels > (grid.h:382, 488)
	const float ml = o.active ? grid_max_level(o, i, F) + 1e-3f : 3.0e38f;
	float x[D], gx[D], res[D];
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) {
		x[d] = pos[(size_t)i * pstride + d];
		gx[d] = gxx[(size_t)i * D + d];
		res[d] = 0.0f;
	}
	for (uint32_t l = 0; l < L; ++l) {
		const LevelInfo li = levels[l];
		float dy[F];
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) dy[f] = dLdy ? (float)dLdy[(size_t)i * dy_stride + l * F + f] : 0.0f;
		float ddy[F];
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) ddy[f] = 0.0f;
		const bool fwd_masked = (float)l >= ml;
		if (interp != Interp::Nearest && !((float)l > ml)) {  // nearest: dy/dx == 0, so every second-order term is 0
			const float s = li.scale;
			float p[D], pd[D], pd2[D];
			uint32_t pg[D];
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) {
				float v = __builtin_fmaf(s, x[d], 0.5f);
				const float t = floorf(v);
				pg[d] = (uint32_t)(int)t;
				v -= t;
				if (interp == Interp::Smoothstep) {
					pd2[d] = __builtin_fmaf(-12.0f, v, 6.0f);
					pd[d] = 6.0f * v * (1.0f - v);
					v = v * v * __builtin_fmaf(-2.0f, v, 3.0f);
				} else {
					pd2[d] = 0.0f;
					pd[d] = 1.0f;
				}
				p[d] = v;
			}
#pragma unroll
			for (uint32_t c = 0; c < (1u << D); ++c) {
				uint32_t local[D];
				float w[D], sg[D];
#pragma unroll
				for (uint32_t d = 0; d < D; ++d) {
					const bool hi = (c >> d) & 1u;
					local[d] = pg[d] + (hi ? 1u : 0u);
					w[d] = hi ? p[d] : 1.0f - p[d];
					sg[d] = hi ? 1.0f : -1.0f;
				}
				const uint32_t idx = (li.offset + grid_index<D, H>(hash_grid != 0, li.size, li.res, local)) * F;
				float A = 0.0f, K[D];
#pragma unroll
				for (uint32_t e = 0; e < D; ++e) {
					float pe = 1.0f;  // prod_{d != e} w_d
#pragma unroll
					for (uint32_t d = 0; d < D; ++d)
						if (d != e) pe *= w[d];
					A += gx[e] * s * pd[e] * sg[e] * pe;
					float k = pd2[e] * gx[e] * sg[e] * pe;
#pragma unroll
					for (uint32_t o = 0; o < D; ++o) {
						if (o == e) continue;
						float po = 1.0f;  // prod_{d != e, o} w_d
#pragma unroll
						for (uint32_t d = 0; d < D; ++d)
							if (d != e && d != o) po *= w[d];
						k += pd[e] * pd[o] * gx[o] * sg[e] * sg[o] * po;
					}
					K[e] = s * s * k;
				}
				float tdy = 0.0f;
#pragma unroll
				for (uint32_t f = 0; f < F; ++f) {
					const float t = (float)table[idx + f];
					ddy[f] += A * t;
					tdy += t * dy[f];
					if (grad && dLdy) unsafeAtomicAdd(grad + idx + f, A * dy[f]);
				}
#pragma unroll
				for (uint32_t e = 0; e < D; ++e) res[e] += K[e] * tdy;
			}
		}
		if (dLddLdy)
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) dLddLdy[(size_t)i * ddy_stride + l * F + f] = (_Float16)(fwd_masked ? 0.0f : ddy[f]);
	}
	if (dLddLdy)
		for (uint32_t k = L * F; k < ddy_stride; ++k) dLddLdy[(size_t)i * ddy_stride + k] = (_Float16)0.0f;
	if (dx)
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) dx[(size_t)i * D + d] = res[d];
}

template <uint32_t D, uint32_t F>
static void grid_bwd_bwd_h(hipStream_t st, HashType h, dim3 g, uint32_t B, uint32_t L, const float* pos, uint32_t ps,
                           const _Float16* t, const float* gx, const _Float16* dy, uint32_t dys, float* grad, _Float16* ddy,
                           uint32_t ddys, float* dx, const LevelInfo* lv, uint32_t hg, uint32_t in, const GridOpts& go) {
#define GBB_LAUNCH(HH) hipLaunchKernelGGL((k_grid_bwd_bwd<D, F, HH>), g, dim3(256), 0, st, B, L, pos, ps, t, gx, dy, dys, grad, ddy, ddys, dx, lv, hg, in, go)
	switch (h) {
		case HashType::Prime: GBB_LAUNCH(HashType::Prime); break;
		case HashType::ReversedPrime: GBB_LAUNCH(HashType::ReversedPrime); break;
		default: GBB_LAUNCH(HashType::CoherentPrime); break;
	}
#undef GBB_LAUNCH
}

template <uint32_t D>
static void grid_bwd_bwd_f(hipStream_t st, uint32_t F, HashType h, dim3 g, uint32_t B, uint32_t L, const float* pos, uint32_t ps,
                           const _Float16* t, const float* gx, const _Float16* dy, uint32_t dys, float* grad, _Float16* ddy,
                           uint32_t ddys, float* dx, const LevelInfo* lv, uint32_t hg, uint32_t in, const GridOpts& go) {
	switch (F) {
		case 1: grid_bwd_bwd_h<D, 1>(st, h, g, B, L, pos, ps, t, gx, dy, dys, grad, ddy, ddys, dx, lv, hg, in, go); break;
		case 2: grid_bwd_bwd_h<D, 2>(st, h, g, B, L, pos, ps, t, gx, dy, dys, grad, ddy, ddys, dx, lv, hg, in, go); break;
		case 4: grid_bwd_bwd_h<D, 4>(st, h, g, B, L, pos, ps, t, gx, dy, dys, grad, ddy, ddys, dx, lv, hg, in, go); break;
		case 8: grid_bwd_bwd_h<D, 8>(st, h, g, B, L, pos, ps, t, gx, dy, dys, grad, ddy, ddys, dx, lv, hg, in, go); break;
		default: throw std::runtime_error("GridEncoding: n_features_per_level must be 1, 2, 4 or 8");
	}
}

void launch_grid_bwd_bwd(hipStream_t st, uint32_t D, uint32_t F, HashType h, uint32_t B, uint32_t L, const float* pos,
                         uint32_t pos_stride, const void* table16, const float* dL_ddLdx, const void* dLdy16, uint32_t dy_stride,
                         float* grad32, void* dLddLdy16, uint32_t ddy_stride, float* dx, const LevelInfo* levels, bool hash_grid,
                         Interp interp, const GridOpts& go) {
	if (B == 0) return;
	const dim3 g(div_round_up(B, 256));
	const _Float16* t = (const _Float16*)table16;
	const _Float16* dy = (const _Float16*)dLdy16;
	_Float16* ddy = (_Float16*)dLddLdy16;
	const uint32_t hg = hash_grid ? 1u : 0u, in = (uint32_t)interp;
	switch (D) {
		case 2: grid_bwd_bwd_f<2>(st, F, h, g, B, L, pos, pos_stride, t, dL_ddLdx, dy, dy_stride, grad32, ddy, ddy_stride, dx, levels, hg, in, go); break;
		case 3: grid_bwd_bwd_f<3>(st, F, h, g, B, L, pos, pos_stride, t, dL_ddLdx, dy, dy_stride, grad32, ddy, ddy_stride, dx, levels, hg, in, go); break;
		case 4: grid_bwd_bwd_f<4>(st, F, h, g, B, L, pos, pos_stride, t, dL_ddLdx, dy, dy_stride, grad32, ddy, ddy_stride, dx, levels, hg, in, go); break;
		default: throw std::runtime_error("GridEncoding: number of input dims must be 2, 3 or 4");
	}
	TCNN_HIP_CHECK(hipGetLastError());
}

struct GridBwdLaunch {
	uint32_t n_items, n_chunks;
	GridBwdEpilogue ep;
	unsigned long long* dbg_times;
	GridOpts opts;
};

// Diagnostic (TCNN_DEBUG_GRID_TIMES=1): per-workgroup start/end wall clock of the grid backward,
// printed per work item to stderr after a synchronising copy. Never set in measured runs.
static DevBufLite g_dbg_times;
static bool dbg_grid_times() {
	static const bool on = std::getenv("TCNN_DEBUG_GRID_TIMES") != nullptr;
	return on;
}

template <uint32_t D, uint32_t F, HashType H>
static void grid_bwd_t(hipStream_t st, int layout, uint32_t dys, dim3 g, size_t lds, uint32_t B, const float* pos, uint32_t ps,
                       const _Float16* dy, const GridSlice* sl, float* part, uint32_t pstr, const LevelInfo* lv,
                       uint32_t hg, uint32_t in, uint32_t ppc, const GridBwdLaunch& gl) {
	// the options (max_level, stochastic) are a separate instantiation: the default kernel stays lean
	static bool attr = false;
	if (!attr) {
		TCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k_grid_bwd_lds<D, F, H, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GRID_BWD_LDS_BYTES));
		TCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k_grid_bwd_lds<D, F, H, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GRID_BWD_LDS_BYTES));
		attr = true;
	}
	if (gl.opts.active)
		hipLaunchKernelGGL((k_grid_bwd_lds<D, F, H, true>), g, dim3(GRID_BWD_THREADS), lds, st, layout, B, pos, ps, dy, dys, sl, part, pstr, lv, hg, in,
		                   ppc, gl.n_items, gl.n_chunks, gl.ep, gl.dbg_times, gl.opts);
	else
		hipLaunchKernelGGL((k_grid_bwd_lds<D, F, H, false>), g, dim3(GRID_BWD_THREADS), lds, st, layout, B, pos, ps, dy, dys, sl, part, pstr, lv, hg, in,
		                   ppc, gl.n_items, gl.n_chunks, gl.ep, gl.dbg_times, gl.opts);
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
static void grid_bwd_f(hipStream_t st, uint32_t F, HashType h, int pairs, uint32_t dys, dim3 g, size_t lds, uint32_t B, const float* pos,
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

void launch_grid_bwd(hipStream_t st, uint32_t D, uint32_t F, HashType h, uint32_t B, const float* pos,
                     uint32_t pos_stride, const void* dLdy16, int dy_layout, uint32_t dy_stride, const GridSlice* slices,
                     uint32_t n_slices, uint32_t n_chunks, float* partial, uint32_t partial_stride,
                     const LevelInfo* levels, bool hash_grid, Interp interp, const GridBwdEpilogue* ep, const GridOpts& go) {
	if (B == 0 || n_slices == 0) return;
	const uint32_t ppc = div_round_up(B, n_chunks);
	GridBwdLaunch gl{};
	gl.n_items = n_slices;
	gl.n_chunks = n_chunks;
	if (ep) gl.ep = *ep;
	else gl.ep.enabled = 0;
	gl.dbg_times = nullptr;
	gl.opts = go;
	const uint32_t n_tail = (ep && ep->enabled) ? ep->n_mlp_groups : 0u;
	dim3 g(n_slices * n_chunks + n_tail);
	if (dbg_grid_times()) gl.dbg_times = (unsigned long long*)g_dbg_times.get((size_t)g.x * 16);
	const size_t lds = GRID_BWD_LDS_BYTES;
	const _Float16* dy = (const _Float16*)dLdy16;
	switch (D) {
		case 2: grid_bwd_f<2>(st, F, h, dy_layout, dy_stride, g, lds, B, pos, pos_stride, dy, slices, partial, partial_stride, levels, hash_grid, (uint32_t)interp, ppc, gl); break;
		case 3: grid_bwd_f<3>(st, F, h, dy_layout, dy_stride, g, lds, B, pos, pos_stride, dy, slices, partial, partial_stride, levels, hash_grid, (uint32_t)interp, ppc, gl); break;
		case 4: grid_bwd_f<4>(st, F, h, dy_layout, dy_stride, g, lds, B, pos, pos_stride, dy, slices, partial, partial_stride, levels, hash_grid, (uint32_t)interp, ppc, gl); break;
		default: throw std::runtime_error("GridEncoding: number of input dims must be 2, 3 or 4");
	}
	TCNN_HIP_CHECK(hipGetLastError());
	if (gl.dbg_times) {
		std::vector<unsigned long long> t((size_t)g.x * 2);
		TCNN_HIP_CHECK(hipStreamSynchronize(st));
		TCNN_HIP_CHECK(hipMemcpy(t.data(), gl.dbg_times, t.size() * 8, hipMemcpyDeviceToHost));
		unsigned long long t0 = ~0ull, t1 = 0;
		for (uint32_t b = 0; b < g.x; ++b) { t0 = std::min(t0, t[2 * b]); t1 = std::max(t1, t[2 * b + 1]); }
		fprintf(stderr, "grid_bwd: %u items x %u chunks + %u tail, span %.1f us\n", n_slices, n_chunks, n_tail, (t1 - t0) / 100.0);
		for (uint32_t it = 0; it < n_slices; ++it) {
			double sum = 0, mx = 0, st0 = 1e30;
			for (uint32_t c = 0; c < n_chunks; ++c) {
				const uint32_t b = c * n_slices + it;
				const double d = (t[2 * b + 1] - t[2 * b]) / 100.0;
				sum += d; mx = std::max(mx, d); st0 = std::min(st0, (t[2 * b] - t0) / 100.0);
			}
			fprintf(stderr, "  item %2u: mean %.1f max %.1f us, first start +%.1f\n", it, sum / n_chunks, mx, st0);
		}
		for (uint32_t b = n_slices * n_chunks; b < g.x; ++b)
			fprintf(stderr, "  tail wg %u: %.1f us start +%.1f\n", b - n_slices * n_chunks, (t[2 * b + 1] - t[2 * b]) / 100.0, (t[2 * b] - t0) / 100.0);
	}
}

}  // namespace tcnn_amd
