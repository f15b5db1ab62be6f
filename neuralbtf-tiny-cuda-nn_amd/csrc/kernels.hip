// kernels.hip -- gfx950 kernels of the hot path + their launchers.
//
//   k_fused_train_grid  grid encode + fused MLP fwd + RelativeL2 + MLP bwd + dW partials (mlp_fused.h)
//   k_grid_fwd          standalone multiresolution grid forward   (reference grid.h:48-212)
//   k_grid_bwd_sliced   grid backward, LDS-privatised per (level, entry slice, point chunk)
//                       (reference grid.h:214-320; fp32 accumulation instead of fp16 atomics)
//   k_reduce_partials   sum of per-workgroup fp32 partial slabs
//   k_adam              Adam (reference optimizers/adam.h:47-119) reading fp32 gradient sums
//   k_relative_l2       standalone RelativeL2 (reference losses/relative_l2.h:40-76)
#include "kernels.h"

#include "grid_device.h"
#include "mlp_fused.h"

namespace tcnn_amd {

// =============================================================================================
// fused train step
// =============================================================================================

#define TCNN_FUSED_SHAPES(X) \
	X(64, 32, 2)             \
	X(64, 32, 1)             \
	X(64, 32, 3)             \
	X(32, 32, 2)             \
	X(32, 32, 1)

bool fused_train_supported(uint32_t W, uint32_t IN, uint32_t NH, uint32_t D, uint32_t F, uint32_t OUTP, int act, HashType h) {
	if (F != 2 || OUTP != 16 || (D != 2 && D != 3) || (act != 0 && act != 1)) return false;
#define X(w, in, nh) if (W == w && IN == in && NH == nh) return true;
	TCNN_FUSED_SHAPES(X)
#undef X
	return false;
}

size_t fused_weight_image_bytes(uint32_t W, uint32_t IN, uint32_t NH) {
#define X(w, in, nh) if (W == w && IN == in && NH == nh) return (size_t)FusedLayout<w, in, nh>::oStage * 2;
	TCNN_FUSED_SHAPES(X)
#undef X
	return 0;
}

void launch_pack_weights(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, const void* params16, void* image) {
#define X(w, in, nh)                                                                                               \
	if (W == w && IN == in && NH == nh) {                                                                          \
		hipLaunchKernelGGL((k_pack_weights<w, in, nh>), dim3(8), dim3(256), 0, st, (const _Float16*)params16, (_Float16*)image); \
		TCNN_HIP_CHECK(hipGetLastError());                                                                         \
		return;                                                                                                    \
	}
	TCNN_FUSED_SHAPES(X)
#undef X
	throw std::runtime_error("pack weights: unsupported shape");
}

static uint32_t device_cu_count() {
	int dev = 0, n = 0;
	TCNN_HIP_CHECK(hipGetDevice(&dev));
	static int cached_dev = -1;
	static uint32_t cached = 0;
	if (dev != cached_dev) {
		TCNN_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
		cached = n > 0 ? (uint32_t)n : 1u;
		cached_dev = dev;
	}
	return cached;
}

// The pipelined 8-wave kernel serves 2D grids whose LDS budget fits and whose targets (<= 3 dims)
// ride the LDS-DMA path; everything else takes the register-gather kernel.
static bool fused_use_pipe(uint32_t W, uint32_t IN, uint32_t NH, uint32_t D, uint32_t dims, bool ext_dout) {
	if (D != 2 || (!ext_dout && dims > 3)) return false;
#define X(w, in, nh) if (W == w && IN == in && NH == nh) return PipeLayout<w, in, nh>::FITS;
	TCNN_FUSED_SHAPES(X)
#undef X
	return false;
}

uint32_t fused_train_n_blocks(uint32_t W, uint32_t IN, uint32_t NH, uint32_t D, uint32_t dims, bool ext_dout, uint32_t B) {
	const uint32_t n_cu = device_cu_count();
	if (fused_use_pipe(W, IN, NH, D, dims, ext_dout)) {
		// one persistent 8-wave workgroup per CU
		const uint32_t nb = div_round_up(B / 32, 8);
		return nb < n_cu ? nb : n_cu;
	}
	// 4 waves x 32 samples per workgroup iteration; 2 workgroups per CU, persistent.
	const uint32_t nb = div_round_up(B, 128);
	return nb < 2 * n_cu ? nb : 2 * n_cu;
}

template <int W, int IN, int NH, uint32_t D, HashType H, Act A, bool EXT>
static void launch_fused_e(hipStream_t st, const FusedTrainArgs& args, uint32_t n_blocks) {
	if constexpr (D == 2 && PipeLayout<W, IN, NH>::FITS) {
		if (EXT || args.dims <= 3) {
			hipLaunchKernelGGL((k_fused_train_pipe<W, IN, NH, H, A, EXT>), dim3(n_blocks), dim3(512), 0, st, args);
			TCNN_HIP_CHECK(hipGetLastError());
			return;
		}
	}
	constexpr size_t bytes = RegKernelLayout<W, IN, NH>::BYTES;
	static bool attr = false;
	if (!attr) {
		TCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k_fused_train_grid<W, IN, NH, D, H, A, EXT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
		attr = true;
	}
	hipLaunchKernelGGL((k_fused_train_grid<W, IN, NH, D, H, A, EXT>), dim3(n_blocks), dim3(256), bytes, st, args);
	TCNN_HIP_CHECK(hipGetLastError());
}

template <int W, int IN, int NH, uint32_t D, HashType H, Act A>
static void launch_fused_t(hipStream_t st, const FusedTrainArgs& args, uint32_t n_blocks) {
	if (args.dout) launch_fused_e<W, IN, NH, D, H, A, true>(st, args, n_blocks);
	else launch_fused_e<W, IN, NH, D, H, A, false>(st, args, n_blocks);
}

template <int W, int IN, int NH>
static void launch_fused_shape(hipStream_t st, uint32_t D, HashType h, int act, const FusedTrainArgs& a, uint32_t nb) {
#define DISPATCH_H(DD, AA)                                                                                   \
	switch (h) {                                                                                          \
		case HashType::Prime: launch_fused_t<W, IN, NH, DD, HashType::Prime, AA>(st, a, nb); break;       \
		case HashType::ReversedPrime: launch_fused_t<W, IN, NH, DD, HashType::ReversedPrime, AA>(st, a, nb); break; \
		default: launch_fused_t<W, IN, NH, DD, HashType::CoherentPrime, AA>(st, a, nb); break;            \
	}
	if (D == 2) {
		if (act == 1) { DISPATCH_H(2, Act::ReLU) } else { DISPATCH_H(2, Act::None) }
	} else {
		if (act == 1) { DISPATCH_H(3, Act::ReLU) } else { DISPATCH_H(3, Act::None) }
	}
#undef DISPATCH_H
}

void launch_fused_train(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, uint32_t D, HashType h, int act,
                        uint32_t B, uint32_t dims, float loss_scale, const void* params16, const void* table16,
                        const float* pos, const float* target, void* out16, void* dLdenc_pairs,
                        float* wgrad_partial, float* loss_partial, const LevelInfo* levels, bool hash_grid,
                        Interp interp, uint32_t n_blocks, const void* dout16, const void* wimage) {
	TCNN_CHECK(B % 32 == 0, "fused train: batch must be a multiple of 32");
	FusedTrainArgs a;
	a.wimage = (const _Float16*)wimage;
	a.dout = (const _Float16*)dout16;
	a.B = B;
	a.dims = dims;
	a.loss_scale = loss_scale;
	a.n_total = (float)(B * dims);
	a.params = (const _Float16*)params16;
	a.table = (const uint32_t*)table16;
	a.pos = pos;
	a.target = target;
	a.out = (_Float16*)out16;
	a.dLdenc = (uint32_t*)dLdenc_pairs;
	a.wgrad_partial = wgrad_partial;
	a.loss_partial = loss_partial;
	a.levels = levels;
	a.hash_grid = hash_grid ? 1u : 0u;
	a.interp = (uint32_t)interp;
#define X(w, in, nh) if (W == w && IN == in && NH == nh) { launch_fused_shape<w, in, nh>(st, D, h, act, a, n_blocks); return; }
	TCNN_FUSED_SHAPES(X)
#undef X
	throw std::runtime_error("fused train: unsupported shape");
}

template <int W, int IN, int NH, Act A, bool SOA>
static void launch_infer_t(hipStream_t st, uint32_t B, const void* wimage, const void* in, void* out) {
	constexpr size_t bytes = (size_t)FusedLayout<W, IN, NH>::oStage * 2;
	static bool attr = false;
	if (!attr) {
		TCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k_mlp_infer<W, IN, NH, A, SOA>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
		attr = true;
	}
	uint32_t nb = div_round_up(B, 64);
	if (nb > 1024) nb = 1024;
	hipLaunchKernelGGL((k_mlp_infer<W, IN, NH, A, SOA>), dim3(nb), dim3(256), bytes, st, B, (const _Float16*)wimage,
	                   (const _Float16*)in, (_Float16*)out);
	TCNN_HIP_CHECK(hipGetLastError());
}

bool mlp_infer_supported(uint32_t W, uint32_t IN, uint32_t NH, uint32_t OUTP, int act) {
	if (OUTP != 16 || (act != 0 && act != 1)) return false;
#define X(w, in, nh) if (W == w && IN == in && NH == nh) return true;
	TCNN_FUSED_SHAPES(X)
#undef X
	return false;
}

void launch_mlp_infer(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, int act, bool soa, uint32_t B,
                      const void* wimage, const void* in16, void* out16) {
	TCNN_CHECK(B % 16 == 0, "mlp inference: batch must be a multiple of 16");
	if (B == 0) return;
#define X(w, in, nh)                                                                                      \
	if (W == w && IN == in && NH == nh) {                                                                 \
		if (act == 1) { if (soa) launch_infer_t<w, in, nh, Act::ReLU, true>(st, B, wimage, in16, out16);   \
		                else launch_infer_t<w, in, nh, Act::ReLU, false>(st, B, wimage, in16, out16); }    \
		else { if (soa) launch_infer_t<w, in, nh, Act::None, true>(st, B, wimage, in16, out16);            \
		       else launch_infer_t<w, in, nh, Act::None, false>(st, B, wimage, in16, out16); }             \
		return;                                                                                           \
	}
	TCNN_FUSED_SHAPES(X)
#undef X
	throw std::runtime_error("mlp inference: unsupported shape");
}

__global__ void k_trim_cast(uint32_t B, uint32_t in_stride, uint32_t n_out, const _Float16* __restrict__ in, float* __restrict__ out) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= B * n_out) return;
	const uint32_t b = i / n_out, o = i % n_out;
	out[i] = (float)in[(size_t)b * in_stride + o];
}

void launch_trim_cast(hipStream_t st, uint32_t B, uint32_t in_stride, uint32_t n_out, const void* in16, float* out) {
	if (!B) return;
	hipLaunchKernelGGL(k_trim_cast, dim3(div_round_up((size_t)B * n_out, 256)), dim3(256), 0, st, B, in_stride, n_out, (const _Float16*)in16, out);
	TCNN_HIP_CHECK(hipGetLastError());
}

void launch_fused_train_profile(hipStream_t st, uint32_t B, uint32_t dims, const void* params16, const void* table16,
                                const float* pos, const float* target, void* dLdenc, float* wgrad_partial,
                                float* loss_partial, const LevelInfo* levels, uint32_t n_blocks, const void* wimage,
                                unsigned long long* prof) {
	TCNN_CHECK(dims <= 3, "phase profile: dims <= 3");
	FusedTrainArgs a{};
	a.wimage = (const _Float16*)wimage;
	a.B = B; a.dims = dims; a.loss_scale = 128.0f; a.n_total = (float)(B * dims);
	a.params = (const _Float16*)params16; a.table = (const uint32_t*)table16; a.pos = pos; a.target = target;
	a.out = nullptr; a.dLdenc = (uint32_t*)dLdenc; a.wgrad_partial = wgrad_partial; a.loss_partial = loss_partial;
	a.levels = levels; a.hash_grid = 1; a.interp = (uint32_t)Interp::Linear; a.dout = nullptr; a.prof = prof;
	hipLaunchKernelGGL((k_fused_train_pipe<64, 32, 2, HashType::CoherentPrime, Act::ReLU, false, true>), dim3(n_blocks), dim3(512), 0, st, a);
	TCNN_HIP_CHECK(hipGetLastError());
}

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

// LDS accumulators are int64 fixed point (2^-40 resolution, +-2^23 range): gfx950 executes LDS
// float atomics (ds_add_f32 / ds_pk_add_f16) at ~195 cycles per wave-instruction per CU but
// ds_add_u64 at ~12 (tools/lds_atomic_bench.hip), and integer sums are order-independent, so the
// gradient is bit-reproducible (the reference's fp16 atomics, grid.h:252-255, are not).
constexpr uint32_t GRID_BWD_THREADS = 1024;
constexpr uint32_t GRID_BWD_LDS_BYTES = 128 * 1024;
constexpr float GRID_FIX_SCALE = 1099511627776.0f;       // 2^40
constexpr double GRID_FIX_INV = 1.0 / 1099511627776.0;  // 2^-40

uint32_t grid_bwd_slice_entries(uint32_t F) { return GRID_BWD_LDS_BYTES / (8 * F); }

__device__ __forceinline__ void lds_add_fix(unsigned long long* acc, float v) {
	const long long iv = (long long)(v * GRID_FIX_SCALE);
	__hip_atomic_fetch_add(acc, (unsigned long long)iv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <uint32_t D, uint32_t F, HashType H, int LAYOUT>
__global__ __launch_bounds__(GRID_BWD_THREADS) void k_grid_bwd_sliced(
	uint32_t B, const float* __restrict__ pos, uint32_t pstride, const _Float16* __restrict__ dLdy, uint32_t dy_stride,
	const GridSlice* __restrict__ slices, float* __restrict__ partial, uint32_t partial_stride,
	const LevelInfo* __restrict__ levels, uint32_t hash_grid, uint32_t interp_u, uint32_t pts_per_chunk) {
	extern __shared__ __attribute__((aligned(16))) unsigned long long acc[];
	const GridSlice sl = slices[blockIdx.x];
	const LevelInfo li = levels[sl.level];
	const uint32_t len = sl.end - sl.begin;
	const Interp interp = (Interp)interp_u;
	for (uint32_t j = threadIdx.x; j < len * F; j += blockDim.x) acc[j] = 0ull;
	__syncthreads();
	const uint32_t i0 = blockIdx.y * pts_per_chunk;
	const uint32_t i1 = min(B, i0 + pts_per_chunk);
	constexpr uint32_t U = 8;  // points in flight per thread
	for (uint32_t base = i0 + threadIdx.x; base < i1; base += U * blockDim.x) {
		float xs[U][D], dy[U][F];
#pragma unroll
		for (uint32_t u = 0; u < U; ++u) {
			const uint32_t i = base + u * blockDim.x;
			const bool ok = i < i1;
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) xs[u][d] = ok ? pos[(size_t)i * pstride + d] : 0.0f;
			if constexpr (LAYOUT == 0) {  // level-major feature pairs [l][i][F]
				HVec<F> v;
				if (ok) v = ((const HVec<F>*)dLdy)[(size_t)sl.level * B + i];
#pragma unroll
				for (uint32_t f = 0; f < F; ++f) dy[u][f] = ok ? (float)v.v[f] : 0.0f;
			} else if constexpr (LAYOUT == 1) {  // SoA [(l*F+f)*B + i] (reference RM layout)
#pragma unroll
				for (uint32_t f = 0; f < F; ++f) dy[u][f] = ok ? (float)dLdy[(size_t)(sl.level * F + f) * B + i] : 0.0f;
			} else {  // AoS [i*stride + l*F + f] (reference CM layout)
#pragma unroll
				for (uint32_t f = 0; f < F; ++f) dy[u][f] = ok ? (float)dLdy[(size_t)i * dy_stride + sl.level * F + f] : 0.0f;
			}
		}
#pragma unroll
		for (uint32_t u = 0; u < U; ++u) {
			if (base + u * blockDim.x >= i1) break;
			float p[D];
			uint32_t pg[D];
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) pos_fract(xs[u][d], li.scale, interp, p[d], pg[d]);
			if (interp == Interp::Nearest) {
				const uint32_t rel = grid_index<D, H>(hash_grid != 0, li.size, li.res, pg) - sl.begin;
				if (rel < len) {
#pragma unroll
					for (uint32_t f = 0; f < F; ++f) lds_add_fix(&acc[rel * F + f], dy[u][f]);
				}
				continue;
			}
#pragma unroll
			for (uint32_t c = 0; c < (1u << D); ++c) {
				float w = 1.0f;
				uint32_t local[D];
#pragma unroll
				for (uint32_t d = 0; d < D; ++d) {
					if ((c & (1u << d)) == 0) { w *= 1.0f - p[d]; local[d] = pg[d]; }
					else { w *= p[d]; local[d] = pg[d] + 1; }
				}
				const uint32_t rel = grid_index<D, H>(hash_grid != 0, li.size, li.res, local) - sl.begin;
				if (rel < len) {
					const float wh = (float)(_Float16)w;
#pragma unroll
					for (uint32_t f = 0; f < F; ++f) lds_add_fix(&acc[rel * F + f], wh * dy[u][f]);
				}
			}
		}
	}
	__syncthreads();
	float* dst = partial + (size_t)blockIdx.y * partial_stride + (size_t)(li.offset + sl.begin) * F;
	for (uint32_t j = threadIdx.x; j < len * F; j += blockDim.x) dst[j] = (float)((double)(long long)acc[j] * GRID_FIX_INV);
}

template <uint32_t D, uint32_t F, HashType H, int LAYOUT>
static void grid_bwd_l(hipStream_t st, dim3 g, size_t lds, uint32_t B, const float* pos, uint32_t ps, const _Float16* dy,
                       uint32_t dys, const GridSlice* sl, float* part, uint32_t pstr, const LevelInfo* lv, uint32_t hg,
                       uint32_t in, uint32_t ppc) {
	static bool attr = false;
	if (!attr) {
		TCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k_grid_bwd_sliced<D, F, H, LAYOUT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GRID_BWD_LDS_BYTES));
		attr = true;
	}
	hipLaunchKernelGGL((k_grid_bwd_sliced<D, F, H, LAYOUT>), g, dim3(GRID_BWD_THREADS), lds, st, B, pos, ps, dy, dys, sl, part, pstr, lv, hg, in, ppc);
}

template <uint32_t D, uint32_t F, HashType H>
static void grid_bwd_t(hipStream_t st, int layout, uint32_t dys, dim3 g, size_t lds, uint32_t B, const float* pos, uint32_t ps,
                       const _Float16* dy, const GridSlice* sl, float* part, uint32_t pstr, const LevelInfo* lv,
                       uint32_t hg, uint32_t in, uint32_t ppc) {
	if (layout == 0) grid_bwd_l<D, F, H, 0>(st, g, lds, B, pos, ps, dy, dys, sl, part, pstr, lv, hg, in, ppc);
	else if (layout == 1) grid_bwd_l<D, F, H, 1>(st, g, lds, B, pos, ps, dy, dys, sl, part, pstr, lv, hg, in, ppc);
	else grid_bwd_l<D, F, H, 2>(st, g, lds, B, pos, ps, dy, dys, sl, part, pstr, lv, hg, in, ppc);
}

template <uint32_t D, uint32_t F>
static void grid_bwd_h(hipStream_t st, HashType h, int pairs, uint32_t dys, dim3 g, size_t lds, uint32_t B, const float* pos, uint32_t ps,
                       const _Float16* dy, const GridSlice* sl, float* part, uint32_t pstr, const LevelInfo* lv,
                       uint32_t hg, uint32_t in, uint32_t ppc) {
	switch (h) {
		case HashType::Prime: grid_bwd_t<D, F, HashType::Prime>(st, pairs, dys, g, lds, B, pos, ps, dy, sl, part, pstr, lv, hg, in, ppc); break;
		case HashType::ReversedPrime: grid_bwd_t<D, F, HashType::ReversedPrime>(st, pairs, dys, g, lds, B, pos, ps, dy, sl, part, pstr, lv, hg, in, ppc); break;
		default: grid_bwd_t<D, F, HashType::CoherentPrime>(st, pairs, dys, g, lds, B, pos, ps, dy, sl, part, pstr, lv, hg, in, ppc); break;
	}
}

template <uint32_t D>
static void grid_bwd_f(hipStream_t st, uint32_t F, HashType h, int pairs, uint32_t dys, dim3 g, size_t lds, uint32_t B, const float* pos,
                       uint32_t ps, const _Float16* dy, const GridSlice* sl, float* part, uint32_t pstr, const LevelInfo* lv,
                       uint32_t hg, uint32_t in, uint32_t ppc) {
	switch (F) {
		case 1: grid_bwd_h<D, 1>(st, h, pairs, dys, g, lds, B, pos, ps, dy, sl, part, pstr, lv, hg, in, ppc); break;
		case 2: grid_bwd_h<D, 2>(st, h, pairs, dys, g, lds, B, pos, ps, dy, sl, part, pstr, lv, hg, in, ppc); break;
		case 4: grid_bwd_h<D, 4>(st, h, pairs, dys, g, lds, B, pos, ps, dy, sl, part, pstr, lv, hg, in, ppc); break;
		case 8: grid_bwd_h<D, 8>(st, h, pairs, dys, g, lds, B, pos, ps, dy, sl, part, pstr, lv, hg, in, ppc); break;
		default: throw std::runtime_error("GridEncoding: n_features_per_level must be 1, 2, 4 or 8");
	}
}

void launch_grid_bwd(hipStream_t st, uint32_t D, uint32_t F, HashType h, uint32_t B, const float* pos,
                     uint32_t pos_stride, const void* dLdy16, int dy_layout, uint32_t dy_stride, const GridSlice* slices,
                     uint32_t n_slices, uint32_t n_chunks, float* partial, uint32_t partial_stride,
                     const LevelInfo* levels, bool hash_grid, Interp interp) {
	if (B == 0 || n_slices == 0) return;
	const uint32_t ppc = div_round_up(B, n_chunks);
	dim3 g(n_slices, n_chunks);
	const size_t lds = (size_t)grid_bwd_slice_entries(F) * F * 8;
	const _Float16* dy = (const _Float16*)dLdy16;
	switch (D) {
		case 2: grid_bwd_f<2>(st, F, h, dy_layout, dy_stride, g, lds, B, pos, pos_stride, dy, slices, partial, partial_stride, levels, hash_grid, (uint32_t)interp, ppc); break;
		case 3: grid_bwd_f<3>(st, F, h, dy_layout, dy_stride, g, lds, B, pos, pos_stride, dy, slices, partial, partial_stride, levels, hash_grid, (uint32_t)interp, ppc); break;
		case 4: grid_bwd_f<4>(st, F, h, dy_layout, dy_stride, g, lds, B, pos, pos_stride, dy, slices, partial, partial_stride, levels, hash_grid, (uint32_t)interp, ppc); break;
		default: throw std::runtime_error("GridEncoding: number of input dims must be 2, 3 or 4");
	}
	TCNN_HIP_CHECK(hipGetLastError());
}

// =============================================================================================
// reductions, Adam, casts, loss
// =============================================================================================

// Sum of fp32 partial slabs, at most two deterministic passes: (param block, part group) -> group
// sums, then groups -> out. Every thread issues 4-wide loads over one group of parts.
__global__ __launch_bounds__(256) void k_reduce_groups(const float* __restrict__ in, uint32_t n_parts, uint32_t group,
                                                        uint32_t stride, uint32_t n, float* __restrict__ out, uint32_t out_stride) {
	const uint32_t p4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
	if (p4 >= n) return;
	const uint32_t j0 = blockIdx.y * group;
	const uint32_t j1 = min(n_parts, j0 + group);
	float* dst = out + (size_t)blockIdx.y * out_stride;
	if (p4 + 4 <= n && (stride % 4) == 0 && (out_stride % 4) == 0) {
		f4 s = {0.0f, 0.0f, 0.0f, 0.0f};
		for (uint32_t j = j0; j < j1; ++j) s += *(const f4*)(in + (size_t)j * stride + p4);
		*(f4*)(dst + p4) = s;
	} else {
		for (uint32_t p = p4; p < n && p < p4 + 4; ++p) {
			float s = 0.0f;
			for (uint32_t j = j0; j < j1; ++j) s += in[(size_t)j * stride + p];
			dst[p] = s;
		}
	}
}

static DevBufLite g_red_tmp;

void launch_reduce_partials(hipStream_t st, const float* in, uint32_t n_parts, uint32_t stride, uint32_t n, float* out) {
	if (n == 0) return;
	constexpr uint32_t MAXG = 16;
	const uint32_t bx = div_round_up(div_round_up(n, 4), 256);
	if (n_parts <= MAXG) {
		hipLaunchKernelGGL(k_reduce_groups, dim3(bx, 1), dim3(256), 0, st, in, n_parts, n_parts, stride, n, out, 0u);
	} else {
		const uint32_t group = div_round_up(n_parts, MAXG);
		const uint32_t G = div_round_up(n_parts, group);
		const uint32_t ostride = (n + 3) / 4 * 4;
		float* tmp = (float*)g_red_tmp.get((size_t)G * ostride * 4);
		hipLaunchKernelGGL(k_reduce_groups, dim3(bx, G), dim3(256), 0, st, in, n_parts, group, stride, n, tmp, ostride);
		TCNN_HIP_CHECK(hipGetLastError());
		hipLaunchKernelGGL(k_reduce_groups, dim3(bx, 1), dim3(256), 0, st, tmp, G, G, ostride, n, out, 0u);
	}
	TCNN_HIP_CHECK(hipGetLastError());
}

// reference optimizers/adam.h:47-119; the fp32 gradient sum is rounded to fp16 first because the
// reference's gradient buffer is __half (trainer.h:327).
__global__ __launch_bounds__(256) void k_adam(const AdamArgs a, float* __restrict__ w32, _Float16* __restrict__ w16,
                                               const float* __restrict__ grad32, _Float16* __restrict__ grad16,
                                               float* __restrict__ m1, float* __restrict__ m2, uint32_t* __restrict__ steps) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= a.n) return;
	const _Float16 g16 = (_Float16)(grad32[i] * a.grad_scale);
	if (grad16) grad16[i] = g16;
	float gradient = (float)g16 / a.loss_scale;
	if (i >= a.n_matrix) {
		if (!a.opt_nonmatrix || gradient == 0.0f) return;
	} else {
		if (!a.opt_matrix) return;
	}
	const float wfp = w32[i];
	if (i < a.n_matrix) gradient = __builtin_fmaf(a.l2_reg, wfp, gradient);
	const float gsq = gradient * gradient;
	const float mm1 = __builtin_fmaf(a.beta1, m1[i], (1.0f - a.beta1) * gradient);
	const float mm2 = __builtin_fmaf(a.beta2, m2[i], (1.0f - a.beta2) * gsq);
	m1[i] = mm1;
	m2[i] = mm2;
	float lr = a.lr;
	if (i >= a.n_matrix) lr *= a.nonmat_lr_factor;
	const uint32_t st = ++steps[i];
	lr *= sqrtf(1.0f - powf(a.beta2, (float)st)) / (1.0f - powf(a.beta1, (float)st));
	const float eff = fminf(fmaxf(lr / (sqrtf(mm2) + a.eps), a.lower_lr_bound), a.upper_lr_bound);
	const float decayed = __builtin_fmaf(1.0f - a.rel_decay * lr, wfp, -copysignf(a.abs_decay * lr, wfp));
	float nw = __builtin_fmaf(-eff, mm1, decayed);
	if (a.clip != 0.0f) nw = fminf(fmaxf(nw, -a.clip), a.clip);
	w32[i] = nw;
	w16[i] = (_Float16)nw;
}

void launch_adam(hipStream_t st, const AdamArgs& a, float* w32, void* w16, const float* grad32, void* grad16,
                 float* m1, float* m2, uint32_t* steps) {
	if (a.n == 0) return;
	hipLaunchKernelGGL(k_adam, dim3(div_round_up(a.n, 256)), dim3(256), 0, st, a, w32, (_Float16*)w16, grad32, (_Float16*)grad16, m1, m2, steps);
	TCNN_HIP_CHECK(hipGetLastError());
}

__global__ void k_cast_f32_f16(const float* __restrict__ in, _Float16* __restrict__ out, size_t n) {
	const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) out[i] = (_Float16)in[i];
}
__global__ void k_cast_f16_f32(const _Float16* __restrict__ in, float* __restrict__ out, size_t n) {
	const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) out[i] = (float)in[i];
}
void launch_cast_f32_f16(hipStream_t st, const float* in, void* out, size_t n) {
	if (!n) return;
	hipLaunchKernelGGL(k_cast_f32_f16, dim3(div_round_up(n, 256)), dim3(256), 0, st, in, (_Float16*)out, n);
	TCNN_HIP_CHECK(hipGetLastError());
}
void launch_cast_f16_f32(hipStream_t st, const void* in, float* out, size_t n) {
	if (!n) return;
	hipLaunchKernelGGL(k_cast_f16_f32, dim3(div_round_up(n, 256)), dim3(256), 0, st, (const _Float16*)in, out, n);
	TCNN_HIP_CHECK(hipGetLastError());
}

__global__ __launch_bounds__(256) void k_relative_l2(uint32_t n_elements, uint32_t stride, uint32_t dims, float loss_scale,
                                                      const _Float16* __restrict__ pred, const float* __restrict__ target,
                                                      float* __restrict__ values, _Float16* __restrict__ grads) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n_elements) return;
	const uint32_t intra = i % stride, inter = i / stride;
	if (intra >= dims) {
		if (values) values[i] = 0.0f;
		grads[i] = (_Float16)0.0f;
		return;
	}
	const float n_total = (float)(n_elements / stride * dims);
	const float p = (float)pred[i];
	const float pse = __builtin_fmaf(p, p, 0.01f);
	const float d = p - target[inter * dims + intra];
	if (values) values[i] = d * d / pse / n_total;
	const float gr = 2.0f * d / pse;
	grads[i] = (_Float16)(loss_scale * gr / n_total);
}

void launch_relative_l2(hipStream_t st, uint32_t B, uint32_t stride, uint32_t dims, float loss_scale,
                        const void* pred16, const float* target, float* values, void* grads16) {
	const uint32_t n = B * stride;
	if (!n) return;
	hipLaunchKernelGGL(k_relative_l2, dim3(div_round_up(n, 256)), dim3(256), 0, st, n, stride, dims, loss_scale,
	                   (const _Float16*)pred16, target, values, (_Float16*)grads16);
	TCNN_HIP_CHECK(hipGetLastError());
}

__global__ __launch_bounds__(256) void k_sum(const float* __restrict__ in, uint32_t n, float* __restrict__ out) {
	__shared__ float part[4];
	float s = 0.0f;
	for (uint32_t i = threadIdx.x; i < n; i += 256) s += in[i];
#pragma unroll
	for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
	if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
	__syncthreads();
	if (threadIdx.x == 0) out[0] = part[0] + part[1] + part[2] + part[3];
}

void launch_sum(hipStream_t st, const float* in, uint32_t n, float* out) {
	hipLaunchKernelGGL(k_sum, dim3(1), dim3(256), 0, st, in, n, out);
	TCNN_HIP_CHECK(hipGetLastError());
}

// =============================================================================================
// layout probe (MFMA f16 operand maps + ds_read_b64_tr_b16), checked by tests/test_gpu_probe.py
// =============================================================================================
__global__ void k_probe(float* mfma_out, int16_t* tr_out) {
	extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
	uint16_t* S = (uint16_t*)smem;
	const int l = threadIdx.x, c = l & 15, q = l >> 4;
	for (int j = l; j < 32 * 24; j += 64) S[j] = (uint16_t)((j / 24) * 64 + (j % 24));
	__syncthreads();
	h8 av, bv;
	for (int e = 0; e < 8; ++e) {
		const int k = 8 * q + e;
		av[e] = (_Float16)(float)(((c * 3 + k * 5) % 11) - 5);  // A[i=c][k]
		bv[e] = (_Float16)(float)(((k * 7 + c * 2) % 13) - 6);  // B[k][j=c]
	}
	const f4 d = mfma16(av, bv, f4{0.0f, 0.0f, 0.0f, 0.0f});
	for (int r = 0; r < 4; ++r) mfma_out[l * 4 + r] = d[r];
	const h8 t = lds_trfrag(smem, 24, q, c, 0);
	*(uint4*)(tr_out + l * 8) = __builtin_bit_cast(uint4, t);
}

__global__ void k_probe_hfma(const h2* a, const h2* b, const h2* c, h2* out, uint32_t n) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) out[i] = pk_fma_f16(a[i], b[i], c[i]);
}

void launch_probe_hfma(hipStream_t st, const void* a, const void* b, const void* c, void* out, uint32_t n_pairs) {
	hipLaunchKernelGGL(k_probe_hfma, dim3(div_round_up(n_pairs, 256)), dim3(256), 0, st, (const h2*)a, (const h2*)b, (const h2*)c, (h2*)out, n_pairs);
	TCNN_HIP_CHECK(hipGetLastError());
}

void launch_probe(hipStream_t st, float* mfma_out, int16_t* tr_out) {
	hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 32 * 24 * 2, st, mfma_out, tr_out);
	TCNN_HIP_CHECK(hipGetLastError());
}

}  // namespace tcnn_amd
