// grid.hip -- multiresolution grid encoding kernels for gfx950:
//   k_grid_fwd      standalone grid forward (reference grid.h:48-212)
//   launch_grid_bwd dispatcher of the LDS-privatised grid backward (grid_bwd_lds.h, one TU per D:
//                   grid_bwd_d{2,3,4}.hip; reference grid.h:214-320, int32 fixed-point sums)
//   k_grid_bwd_input, k_grid_bwd_bwd  input / second-order gradients (grid.h:322-650)
#include "kernels.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "adam_device.h"
#include "grid_bwd_lds.h"
#include "grid_device.h"

namespace tcnn_amd {
// =============================================================================================
// grid forward (standalone)
// =============================================================================================

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
		float wf[NC];
#pragma unroll
		for (uint32_t c = 0; c < NC; ++c) {
			float w = 1.0f;
			uint32_t local[D];
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) {
				if ((c & (1u << d)) == 0) { w *= 1.0f - p[d]; local[d] = pg[d]; }
				else { w *= p[d]; local[d] = pg[d] + 1; }
			}
			wf[c] = w;  // converted in pairs, see encode_level_f2 (tests/test_isa_rounding.py)
			v[c] = tv[li.offset + grid_index<D, H>(hash_grid != 0, li.size, li.res, local)];
		}
		f16_rn_pairs(wf, w16);
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

// AoS forward for F = 2 (the trainer's encoding pass of the tile / layer-wise engines): one
// workgroup = 64 consecutive points x all levels; wave w encodes levels w, w+4, ... for the 64
// points, so a level is wave-uniform (scalar LevelInfo loads, no divergence between dense and
// hashed index math, and the 64 lanes' gathers of a coarse level share cache lines), and the
// [64][L] half2 tile is transposed through LDS into whole 16-byte output rows.
template <uint32_t D, HashType H>
__global__ __launch_bounds__(256) void k_grid_fwd_aos_f2(uint32_t B, const float* __restrict__ pos, uint32_t pstride,
                                                         const uint32_t* __restrict__ table, _Float16* __restrict__ out,
                                                         uint32_t out_stride, const LevelInfo* __restrict__ levels, uint32_t hash_grid,
                                                         uint32_t interp_u, const GridOpts o, uint32_t L) {
	__shared__ uint32_t tile[64 * 65];  // [point][level], row stride 65 (conflict-free column writes)
	const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
	const uint32_t i = blockIdx.x * 64 + lane;
	const bool valid = i < B;
	const Interp interp = (Interp)interp_u;
	float x[D];
	bool inr = true;
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) {
		x[d] = valid ? pos[(size_t)i * pstride + d] : 0.0f;
		inr = inr && x[d] >= 0.0f && x[d] <= 1.0f;
	}
	// all 64 points in [0, 1]: the branch-free index (see grid_index_inrange)
	const bool fast = o.inrange_index && !o.active && __builtin_amdgcn_ballot_w64(!inr) == 0;
	if (fast) {
		// four levels per wave at a time with all their gathers in flight together (a level past L
		// encodes level 0 into a discarded register, so the body has no branch to split the batch);
		// lanes L, L^1 (neighbouring points, same level) fetch each other's x-neighbour corners in one
		// instruction (encode_level_f2_pair)
		const uint32_t par = lane & 1u;
		float xA[D], xB[D];
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) {
			const float ox = dpp_swap_pair(x[d]);
			xA[d] = par ? ox : x[d];
			xB[d] = par ? x[d] : ox;
		}
		for (uint32_t l0 = 0; l0 < L; l0 += 16) {
			h2 r[4];
#pragma unroll
			for (uint32_t k = 0; k < 4; ++k) {
				const uint32_t level = l0 + wave + 4 * k;
				r[k] = encode_level_f2_pair<D, H>(table, level_consts<D>(levels[level < L ? level : 0], hash_grid != 0), xA, xB, par);
			}
#pragma unroll
			for (uint32_t k = 0; k < 4; ++k) {
				const uint32_t level = l0 + wave + 4 * k;
				if (level < L) tile[lane * 65 + level] = valid ? __builtin_bit_cast(uint32_t, r[k]) : 0u;
			}
		}
	}
	for (uint32_t level = fast ? L : wave; level < L; level += 4) {
		const LevelInfo li = levels[level];
		h2 r = {(_Float16)0.0f, (_Float16)0.0f};
		if (valid && !(o.active && (float)level >= grid_max_level(o, i, 2) + 1e-3f)) {  // masked: 0 (grid.h:75-91)
			r = encode_level_f2<D, H>(table, li, hash_grid != 0, interp, x);
		}
		tile[lane * 65 + level] = __builtin_bit_cast(uint32_t, r);
	}
	__syncthreads();
	const uint32_t row2 = out_stride / 2;  // half2 columns per output row (grid features + zero padding)
	uint32_t* o32 = (uint32_t*)out;
	for (uint32_t idx = threadIdx.x; idx < 64 * row2; idx += 256) {
		const uint32_t p = idx / row2, c2 = idx % row2;
		const uint32_t ip = blockIdx.x * 64 + p;
		if (ip < B) o32[(size_t)ip * row2 + c2] = c2 < L ? tile[p * 65 + c2] : 0u;
	}
}

// SoA forward for F = 2 (the Module forward's kept encoding and the fused inference's input, [L*2][B]
// feature planes): one thread per point for 4 consecutive levels (blockIdx.y), the position loaded
// once and the 4 levels' 16 gathers in flight together; a level is block-uniform. Points of a wave all
// in [0, 1] take the branch-free index (grid_index_inrange, as k_grid_fwd_aos_f2), any other wave the
// generic index. Same values as k_grid_fwd (encode_level_f2: the reference's fp16 FMA chain).
template <uint32_t D, HashType H>
__global__ __launch_bounds__(256) void k_grid_fwd_soa_f2(uint32_t B, const float* __restrict__ pos, uint32_t pstride,
                                                         const uint32_t* __restrict__ table, _Float16* __restrict__ out,
                                                         const LevelInfo* __restrict__ levels, uint32_t hash_grid, uint32_t interp_u,
                                                         const GridOpts o, uint32_t L) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	const bool valid = i < B;
	const Interp interp = (Interp)interp_u;
	float x[D];
	bool inr = true;
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) {
		x[d] = valid ? pos[(size_t)i * pstride + d] : 0.0f;
		inr = inr && x[d] >= 0.0f && x[d] <= 1.0f;
	}
	const bool fast = o.inrange_index && !o.active && __builtin_amdgcn_ballot_w64(!inr) == 0;
	const uint32_t l0 = blockIdx.y * 4;
	h2 r[4];
	if (fast) {
		// lanes L, L^1 (neighbouring points) share their gathers' lines (encode_level_f2_pair)
		const uint32_t par = threadIdx.x & 1u;
		float xA[D], xB[D];
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) {
			const float ox = dpp_swap_pair(x[d]);
			xA[d] = par ? ox : x[d];
			xB[d] = par ? x[d] : ox;
		}
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k) {
			const uint32_t level = l0 + k;
			r[k] = encode_level_f2_pair<D, H>(table, level_consts<D>(levels[level < L ? level : 0], hash_grid != 0), xA, xB, par);
		}
	} else {
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k) {
			const uint32_t level = l0 + k;
			r[k] = h2{(_Float16)0.0f, (_Float16)0.0f};
			if (level < L && valid && !(o.active && (float)level >= grid_max_level(o, i, 2) + 1e-3f))  // masked: 0 (grid.h:75-91)
				r[k] = encode_level_f2<D, H>(table, levels[level], hash_grid != 0, interp, x);
		}
	}
	if (!valid) return;
#pragma unroll
	for (uint32_t k = 0; k < 4; ++k) {
		const uint32_t level = l0 + k;
		if (level < L) {
			out[(size_t)(2 * level) * B + i] = r[k][0];
			out[(size_t)(2 * level + 1) * B + i] = r[k][1];
		}
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
	if (!soa && F == 2 && L <= 64 && out_stride % 2 == 0 && interp != Interp::Nearest) {
		const dim3 g2(div_round_up(B, 64));
		const uint32_t* t32 = (const uint32_t*)table16;
		_Float16* o16 = (_Float16*)out16;
		const uint32_t hg = hash_grid ? 1u : 0u, in = (uint32_t)interp;
#define AOS2(DD)                                                                                                                   \
	switch (h) {                                                                                                                   \
		case HashType::Prime: hipLaunchKernelGGL((k_grid_fwd_aos_f2<DD, HashType::Prime>), g2, dim3(256), 0, st, B, pos, pos_stride, t32, o16, out_stride, levels, hg, in, go, L); break; \
		case HashType::ReversedPrime: hipLaunchKernelGGL((k_grid_fwd_aos_f2<DD, HashType::ReversedPrime>), g2, dim3(256), 0, st, B, pos, pos_stride, t32, o16, out_stride, levels, hg, in, go, L); break; \
		default: hipLaunchKernelGGL((k_grid_fwd_aos_f2<DD, HashType::CoherentPrime>), g2, dim3(256), 0, st, B, pos, pos_stride, t32, o16, out_stride, levels, hg, in, go, L); break; \
	}
		if (D == 2) { AOS2(2) }
		else if (D == 3) { AOS2(3) }
		else if (D == 4) { AOS2(4) }
		else throw std::runtime_error("GridEncoding: number of input dims must be 2, 3 or 4");
#undef AOS2
		TCNN_HIP_CHECK(hipGetLastError());
		return;
	}
	if (soa && F == 2 && interp != Interp::Nearest) {
		const dim3 g4(div_round_up(B, 256), div_round_up(L, 4));
		const uint32_t* t32 = (const uint32_t*)table16;
		_Float16* o16 = (_Float16*)out16;
		const uint32_t hg = hash_grid ? 1u : 0u, in = (uint32_t)interp;
#define SOA2(DD)                                                                                                                   \
	switch (h) {                                                                                                                   \
		case HashType::Prime: hipLaunchKernelGGL((k_grid_fwd_soa_f2<DD, HashType::Prime>), g4, dim3(256), 0, st, B, pos, pos_stride, t32, o16, levels, hg, in, go, L); break; \
		case HashType::ReversedPrime: hipLaunchKernelGGL((k_grid_fwd_soa_f2<DD, HashType::ReversedPrime>), g4, dim3(256), 0, st, B, pos, pos_stride, t32, o16, levels, hg, in, go, L); break; \
		default: hipLaunchKernelGGL((k_grid_fwd_soa_f2<DD, HashType::CoherentPrime>), g4, dim3(256), 0, st, B, pos, pos_stride, t32, o16, levels, hg, in, go, L); break; \
	}
		if (D == 2) { SOA2(2) }
		else if (D == 3) { SOA2(3) }
		else if (D == 4) { SOA2(4) }
		else throw std::runtime_error("GridEncoding: number of input dims must be 2, 3 or 4");
#undef SOA2
		TCNN_HIP_CHECK(hipGetLastError());
		return;
	}
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
			for (uint32_t f = 0; f < F; ++f) dLddLdy[(size_t)i * ddy_stride + l * F + f] = f16_rn(fwd_masked ? 0.0f : ddy[f]);
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

// Diagnostic (TCNN_DEBUG_GRID_TIMES=1): per-workgroup start/end wall clock of the grid backward,
// printed per work item to stderr after a synchronising copy. Never set in measured runs.
static DevBufLite g_dbg_times;
static bool dbg_grid_times() {
	static const bool on = std::getenv("TCNN_DEBUG_GRID_TIMES") != nullptr;
	return on;
}

uint32_t grid_bwd_slot_budget() { return GRID_BWD_SLOTS; }

extern template void grid_bwd_f<2>(hipStream_t, uint32_t, HashType, int, uint32_t, dim3, size_t, uint32_t, const float*, uint32_t,
                                   const _Float16*, const GridSlice*, float*, uint32_t, const LevelInfo*, uint32_t, uint32_t, uint32_t,
                                   const GridBwdLaunch&);
extern template void grid_bwd_f<3>(hipStream_t, uint32_t, HashType, int, uint32_t, dim3, size_t, uint32_t, const float*, uint32_t,
                                   const _Float16*, const GridSlice*, float*, uint32_t, const LevelInfo*, uint32_t, uint32_t, uint32_t,
                                   const GridBwdLaunch&);
extern template void grid_bwd_f<4>(hipStream_t, uint32_t, HashType, int, uint32_t, dim3, size_t, uint32_t, const float*, uint32_t,
                                   const _Float16*, const GridSlice*, float*, uint32_t, const LevelInfo*, uint32_t, uint32_t, uint32_t,
                                   const GridBwdLaunch&);

void launch_grid_bwd(hipStream_t st, uint32_t D, uint32_t F, HashType h, uint32_t B, const float* pos,
                     uint32_t pos_stride, const void* dLdy16, int dy_layout, uint32_t dy_stride, const GridSlice* slices,
                     uint32_t n_slices, uint32_t n_chunks, float* partial, uint32_t partial_stride,
                     const LevelInfo* levels, bool hash_grid, Interp interp, const GridBwdEpilogue* ep, const GridOpts& go,
                     const GridSlice* host_slices, const LevelInfo* host_levels, uint32_t n_levels) {
	const uint32_t n_tail = (ep && ep->enabled) ? ep->n_mlp_groups : 0u;
	if (n_tail == 0 && (n_slices == 0 || B == 0)) return;  // callers zero the gradient of empty batches
	if (B == 0) n_slices = 0;
	const uint32_t ppc = div_round_up(std::max(B, 1u), n_chunks);
	GridBwdLaunch gl{};
	gl.n_items = n_slices;
	gl.n_chunks = n_chunks;
	if (ep) gl.ep = *ep;
	else gl.ep.enabled = 0;
	gl.dbg_times = nullptr;
	gl.opts = go;
	gl.tb.n_items = gl.tb.n_levels = 0;
	if (host_slices && host_levels && n_slices <= GRID_BWD_ARG_ITEMS && n_levels <= GRID_BWD_ARG_LEVELS) {
		gl.tb.n_items = n_slices;
		gl.tb.n_levels = n_levels;
		std::copy(host_slices, host_slices + n_slices, gl.tb.items);
		std::copy(host_levels, host_levels + n_levels, gl.tb.levels);
	}
	dim3 g(n_slices * n_chunks + n_tail);
	if (dbg_grid_times()) gl.dbg_times = (unsigned long long*)g_dbg_times.get((size_t)g.x * 64);
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
		std::vector<unsigned long long> t((size_t)g.x * 8);
		TCNN_HIP_CHECK(hipStreamSynchronize(st));
		TCNN_HIP_CHECK(hipMemcpy(t.data(), gl.dbg_times, t.size() * 8, hipMemcpyDeviceToHost));
		unsigned long long t0 = ~0ull, t1 = 0;
		for (uint32_t b = 0; b < g.x; ++b) { t0 = std::min(t0, t[8 * b]); t1 = std::max(t1, t[8 * b + 4]); }
		fprintf(stderr, "grid_bwd: %u items x %u chunks + %u tail, span %.1f us\n", n_slices, n_chunks, n_tail, (t1 - t0) / 100.0);
		for (uint32_t it = 0; it < n_slices; ++it) {
			double sum = 0, mx = 0, st0 = 1e30, ph[4] = {0, 0, 0, 0}, ld = 0, zr = 0;
			for (uint32_t c = 0; c < n_chunks; ++c) {
				const uint32_t b = it * n_chunks + c;
				const double d = (t[8 * b + 4] - t[8 * b]) / 100.0;
				sum += d; mx = std::max(mx, d); st0 = std::min(st0, (t[8 * b] - t0) / 100.0);
				for (int k = 0; k < 4; ++k) ph[k] += (t[8 * b + k + 1] - t[8 * b + k]) / 100.0 / n_chunks;
					ld += ((double)t[8 * b + 5] - (double)t[8 * b]) / 100.0 / n_chunks;
					zr += ((double)t[8 * b + 6] - (double)t[8 * b]) / 100.0 / n_chunks;
			}
			fprintf(stderr, "  item %2u: mean %.1f max %.1f us, first start +%.1f | prepass %.1f (zero %.1f, +loads %.1f) accumulate %.1f merge %.1f write %.1f\n", it,
			        sum / n_chunks, mx, st0, ph[0], zr, ld, ph[1], ph[2], ph[3]);
		}
		for (uint32_t b = n_slices * n_chunks; b < g.x; ++b)
			fprintf(stderr, "  tail wg %u: %.1f us start +%.1f\n", b - n_slices * n_chunks, (t[8 * b + 4] - t[8 * b]) / 100.0, (t[8 * b] - t0) / 100.0);
	}
}

}  // namespace tcnn_amd
