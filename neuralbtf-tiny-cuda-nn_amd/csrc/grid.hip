// grid.hip -- multiresolution grid encoding kernels for gfx950:
//   k_grid_fwd      standalone grid forward (reference grid.h:48-212)
//   k_grid_bwd_lds  grid backward, LDS-privatised per (level, entries x features, point chunk)
//                   (reference grid.h:214-320; int32 fixed-point sums instead of fp16 atomics)
#include "kernels.h"

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
                                                  uint32_t hash_grid, uint32_t interp_u) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= B) return;
	const uint32_t level = blockIdx.y;
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
	if (interp == Interp::Nearest) {
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
                       _Float16* o, uint32_t soa, uint32_t os, const LevelInfo* lv, uint32_t hg, uint32_t in) {
	switch (h) {
		case HashType::Prime: hipLaunchKernelGGL((k_grid_fwd<D, F, HashType::Prime>), g, dim3(256), 0, st, B, pos, ps, t, o, soa, os, lv, hg, in); break;
		case HashType::ReversedPrime: hipLaunchKernelGGL((k_grid_fwd<D, F, HashType::ReversedPrime>), g, dim3(256), 0, st, B, pos, ps, t, o, soa, os, lv, hg, in); break;
		default: hipLaunchKernelGGL((k_grid_fwd<D, F, HashType::CoherentPrime>), g, dim3(256), 0, st, B, pos, ps, t, o, soa, os, lv, hg, in); break;
	}
}

template <uint32_t D>
static void grid_fwd_f(hipStream_t st, uint32_t F, HashType h, dim3 g, uint32_t B, const float* pos, uint32_t ps,
                       const _Float16* t, _Float16* o, uint32_t soa, uint32_t os, const LevelInfo* lv, uint32_t hg, uint32_t in) {
	switch (F) {
		case 1: grid_fwd_h<D, 1>(st, h, g, B, pos, ps, t, o, soa, os, lv, hg, in); break;
		case 2: grid_fwd_h<D, 2>(st, h, g, B, pos, ps, t, o, soa, os, lv, hg, in); break;
		case 4: grid_fwd_h<D, 4>(st, h, g, B, pos, ps, t, o, soa, os, lv, hg, in); break;
		case 8: grid_fwd_h<D, 8>(st, h, g, B, pos, ps, t, o, soa, os, lv, hg, in); break;
		default: throw std::runtime_error("GridEncoding: n_features_per_level must be 1, 2, 4 or 8");
	}
}

void launch_grid_fwd(hipStream_t st, uint32_t D, uint32_t F, HashType h, uint32_t B, uint32_t L,
                     const float* pos, uint32_t pos_stride, const void* table16, void* out16, bool soa,
                     uint32_t out_stride, const LevelInfo* levels, bool hash_grid, Interp interp) {
	if (B == 0) return;
	dim3 g(div_round_up(B, 256), L);
	const _Float16* t = (const _Float16*)table16;
	_Float16* o = (_Float16*)out16;
	switch (D) {
		case 2: grid_fwd_f<2>(st, F, h, g, B, pos, pos_stride, t, o, soa, out_stride, levels, hash_grid, (uint32_t)interp); break;
		case 3: grid_fwd_f<3>(st, F, h, g, B, pos, pos_stride, t, o, soa, out_stride, levels, hash_grid, (uint32_t)interp); break;
		case 4: grid_fwd_f<4>(st, F, h, g, B, pos, pos_stride, t, o, soa, out_stride, levels, hash_grid, (uint32_t)interp); break;
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
template <uint32_t D, uint32_t F, HashType H, int KIND, int MODE>
__device__ __forceinline__ void grid_bwd_points(int layout, uint32_t B, const float* __restrict__ pos, uint32_t pstride,
                                                const _Float16* __restrict__ dLdy, uint32_t dy_stride, uint32_t level,
                                                const LevelInfo& li, bool hash_grid, Interp interp, uint32_t begin,
                                                uint32_t len, uint32_t f0, uint32_t i0, uint32_t i1, float scale, int* acc) {
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
#pragma unroll
			for (uint32_t c = 0; c < (1u << D); ++c) {
				if (nearest && c > 0) break;
				float w = 1.0f;
				uint32_t local[D];
#pragma unroll
				for (uint32_t d = 0; d < D; ++d) {
					if ((c & (1u << d)) == 0) { w *= 1.0f - p[d]; local[d] = pg[d]; }
					else { w *= p[d]; local[d] = pg[d] + 1; }
				}
				const float wh = nearest ? 1.0f : (float)(_Float16)w;
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

template <uint32_t D, uint32_t F, HashType H, int KIND>
__device__ __forceinline__ void grid_bwd_mode(int mode, int layout, uint32_t B, const float* pos, uint32_t pstride,
                                              const _Float16* dLdy, uint32_t dy_stride, uint32_t level, const LevelInfo& li,
                                              bool hash_grid, Interp interp, uint32_t begin, uint32_t len, uint32_t f0,
                                              uint32_t i0, uint32_t i1, float scale, int* acc) {
	if constexpr (F == 2) {
		if (mode == 0) { grid_bwd_points<D, F, H, KIND, 0>(layout, B, pos, pstride, dLdy, dy_stride, level, li, hash_grid, interp, begin, len, f0, i0, i1, scale, acc); return; }
	} else if constexpr (F > 2) {
		if (mode == 2) { grid_bwd_points<D, F, H, KIND, 2>(layout, B, pos, pstride, dLdy, dy_stride, level, li, hash_grid, interp, begin, len, f0, i0, i1, scale, acc); return; }
	}
	grid_bwd_points<D, F, H, KIND, 1>(layout, B, pos, pstride, dLdy, dy_stride, level, li, hash_grid, interp, begin, len, f0, i0, i1, scale, acc);
}

// Network-gradient tail of the epilogue (extra workgroups g = 0 .. n_mlp_groups-1): group sums of
// the fused kernel's slabs (same grouping and order as launch_reduce_partials), then the last
// group finishes the sum, runs Adam on the network parameters and writes the fused weight image.
__device__ void grid_bwd_mlp_tail(const GridBwdEpilogue& ep, uint32_t g, volatile uint32_t* flag) {
	const uint32_t G = ep.n_mlp_groups, N = ep.n_mlp, P = ep.n_wparts;
	const uint32_t per = (P + G - 1) / G;
	const uint32_t j0 = g * per, j1 = min(P, j0 + per);
	float* dst = ep.group_slab + (size_t)g * (N + 4);
	for (uint32_t c = threadIdx.x * 4; c < N; c += blockDim.x * 4)
		*(f4*)(dst + c) = slab_sum((const f4*)(ep.wpart + (size_t)j0 * N + c), N / 4, j1 - j0);
	if (threadIdx.x == 0) {
		float l = 0.0f;
		for (uint32_t j = j0; j < j1; ++j) l += ep.lpart[j];
		dst[N] = l;
	}
	if (!arrive_last(ep.tail_counter, G, flag)) return;
	if (threadIdx.x == 0 && ep.factor_out) *ep.factor_out = adam_bias_factor(ep.adam_mlp, ep.factor_step);
	const uint32_t nW0 = ep.W * ep.IN, nWh = (ep.NH - 1) * ep.W * ep.W;
	for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) {
		const float s = slab_sum(ep.group_slab + i, N + 4, G);
		ep.buf.g32[i] = s;
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
	if (threadIdx.x == 0) {
		float l = 0.0f;
		for (uint32_t k = 0; k < G; ++k) l += ep.group_slab[(size_t)k * (N + 4) + N];
		*ep.d_loss = l;
	}
}

template <uint32_t D, uint32_t F, HashType H>
__global__ __launch_bounds__(GRID_BWD_THREADS) void k_grid_bwd_lds(
	int layout, uint32_t B, const float* __restrict__ pos, uint32_t pstride, const _Float16* __restrict__ dLdy, uint32_t dy_stride,
	const GridSlice* __restrict__ items, float* __restrict__ partial, uint32_t partial_stride,
	const LevelInfo* __restrict__ levels, uint32_t hash_grid, uint32_t interp_u, uint32_t pts_per_chunk, uint32_t n_items,
	uint32_t n_chunks, const GridBwdEpilogue ep) {
	extern __shared__ __attribute__((aligned(16))) int acc[];
	__shared__ float red[GRID_BWD_THREADS / 64];
	volatile uint32_t* flag = (volatile uint32_t*)&red[0];
	if (blockIdx.x >= n_items * n_chunks) {
		grid_bwd_mlp_tail(ep, blockIdx.x - n_items * n_chunks, flag);
		return;
	}
	const uint32_t item = blockIdx.x % n_items, chunk = blockIdx.x / n_items;
	const GridSlice it = items[item];
	const LevelInfo li = levels[it.level];
	const uint32_t len = it.end - it.begin;
	const uint32_t nf = it.nf, f0 = it.f0;
	const Interp interp = (Interp)interp_u;
	for (uint32_t j = threadIdx.x; j < len * nf; j += blockDim.x) acc[j] = 0;
	const uint32_t i0 = chunk * pts_per_chunk;
	const uint32_t i1 = min(B, i0 + pts_per_chunk);

	// pre-pass: max |dL/dy| of this item's features over the chunk -> fixed-point scale
	float m = 0.0f;
	for (uint32_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
		float dy[F];
		load_dy<F>(layout, dLdy, dy_stride, it.level, B, i, dy);
#pragma unroll
		for (uint32_t f = 0; f < F; ++f)
			if (f - f0 < nf) m = fmaxf(m, fabsf(dy[f]));
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
		grid_bwd_mode<D, F, H, IDX_HASH_POW2>(mode, layout, B, pos, pstride, dLdy, dy_stride, it.level, li, hash_grid != 0, interp, it.begin, len, f0, i0, i1, scale, acc);
	else if (kind == IDX_DENSE)
		grid_bwd_mode<D, F, H, IDX_DENSE>(mode, layout, B, pos, pstride, dLdy, dy_stride, it.level, li, hash_grid != 0, interp, it.begin, len, f0, i0, i1, scale, acc);
	else
		grid_bwd_mode<D, F, H, IDX_GENERIC>(mode, layout, B, pos, pstride, dLdy, dy_stride, it.level, li, hash_grid != 0, interp, it.begin, len, f0, i0, i1, scale, acc);
	__syncthreads();
	const float inv = ldexpf(1.0f, -e);
	float* dst = partial + (size_t)chunk * partial_stride + (size_t)(li.offset + it.begin) * F + f0;
	if (mode == 0) {  // decode the packed int32 pairs
		const long long* a64 = (const long long*)acc;
		for (uint32_t j = threadIdx.x; j < len; j += blockDim.x) {
			const long long t = a64[j];
			const int lo = (int)(uint32_t)(unsigned long long)t;
			const int hi = (int)((t - (long long)lo) >> 32);
			*(float2*)(dst + 2 * j) = make_float2((float)lo * inv, (float)hi * inv);
		}
	} else if (nf == F) {
		for (uint32_t j = threadIdx.x; j < len * F; j += blockDim.x) dst[j] = (float)acc[j] * inv;
	} else {
		for (uint32_t j = threadIdx.x; j < len * nf; j += blockDim.x) dst[(j / nf) * F + (j % nf)] = (float)acc[j] * inv;
	}
}

struct GridBwdLaunch {
	uint32_t n_items, n_chunks;
	GridBwdEpilogue ep;
};

template <uint32_t D, uint32_t F, HashType H>
static void grid_bwd_t(hipStream_t st, int layout, uint32_t dys, dim3 g, size_t lds, uint32_t B, const float* pos, uint32_t ps,
                       const _Float16* dy, const GridSlice* sl, float* part, uint32_t pstr, const LevelInfo* lv,
                       uint32_t hg, uint32_t in, uint32_t ppc, const GridBwdLaunch& gl) {
	static bool attr = false;
	if (!attr) {
		TCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k_grid_bwd_lds<D, F, H>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GRID_BWD_LDS_BYTES));
		attr = true;
	}
	hipLaunchKernelGGL((k_grid_bwd_lds<D, F, H>), g, dim3(GRID_BWD_THREADS), lds, st, layout, B, pos, ps, dy, dys, sl, part, pstr, lv, hg, in, ppc,
	                   gl.n_items, gl.n_chunks, gl.ep);
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
                     const LevelInfo* levels, bool hash_grid, Interp interp, const GridBwdEpilogue* ep) {
	if (B == 0 || n_slices == 0) return;
	const uint32_t ppc = div_round_up(B, n_chunks);
	GridBwdLaunch gl{};
	gl.n_items = n_slices;
	gl.n_chunks = n_chunks;
	if (ep) gl.ep = *ep;
	else gl.ep.enabled = 0;
	const uint32_t n_tail = (ep && ep->enabled) ? ep->n_mlp_groups : 0u;
	dim3 g(n_slices * n_chunks + n_tail);
	const size_t lds = GRID_BWD_LDS_BYTES;
	const _Float16* dy = (const _Float16*)dLdy16;
	switch (D) {
		case 2: grid_bwd_f<2>(st, F, h, dy_layout, dy_stride, g, lds, B, pos, pos_stride, dy, slices, partial, partial_stride, levels, hash_grid, (uint32_t)interp, ppc, gl); break;
		case 3: grid_bwd_f<3>(st, F, h, dy_layout, dy_stride, g, lds, B, pos, pos_stride, dy, slices, partial, partial_stride, levels, hash_grid, (uint32_t)interp, ppc, gl); break;
		case 4: grid_bwd_f<4>(st, F, h, dy_layout, dy_stride, g, lds, B, pos, pos_stride, dy, slices, partial, partial_stride, levels, hash_grid, (uint32_t)interp, ppc, gl); break;
		default: throw std::runtime_error("GridEncoding: number of input dims must be 2, 3 or 4");
	}
	TCNN_HIP_CHECK(hipGetLastError());
}

}  // namespace tcnn_amd
