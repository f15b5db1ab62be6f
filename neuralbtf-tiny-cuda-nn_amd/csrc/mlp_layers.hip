// mlp_layers.hip -- layer-wise MFMA MLP engine for gfx950: widths 16, 32, 64, 128, any
// depth, any input width multiple of 16 up to 128, every activation of the reference.
//
// Used for the shapes the register-resident fused kernel (mlp_fused.h) does not cover: W = 128 (the
// LDS-pressure configs: OneBlob W128/H5 = 168 KB of fp16 weights does not fit 160 KB of LDS at all),
// non-grid encodings (OneBlob, Identity), CutlassMLP / "MLP" otypes, output activations.
// Reference: FullyFusedMLP forward/backward (fully_fused_mlp.cu:47-557, 735-836) and CutlassMLP
// (cutlass_mlp.cu:38-371) -- same dataflow as the reference (per-layer fp16 activations in HBM,
// split-K weight-gradient GEMMs), with fp32 MFMA accumulation instead of fp16 accumulators.
//
// Layouts: activations are sample-major AoS [B][width] fp16 (the reference's CM matrices);
// weights row-major [n_out][n_in] fp16 inside the parameter buffer.
//
//   k_layer_fwd<NT, KS>  Y = act(X W^T)               out tiles NT x 16, contraction K <= 32 KS
//   k_layer_bwd<NT, KS>  dX = act'(H) . (dY W)        out tiles NT x 16 over K, contraction N <= 32 KS
//   k_wgrad<MT, KT>      dW partial = dY^T X over a sample chunk (samples on the MFMA K axis,
//                        staged through LDS and read back with ds_read_b64_tr_b16)
//   k_relative_l2_partial RelativeL2 with per-workgroup loss partial sums
#include "kernels.h"

#include <type_traits>

#include "mlp_fused.h"

namespace tcnn_amd {

// Stage a row-major [rows][cols] fp16 matrix into LDS with row stride rs, zero-filling columns
// [cols, zc) (transpose = false), or its transpose [cols][rows] with columns [rows, zc) zeroed.
// Untransposed rows go 8 halves (16 B) per load when cols % 8 == 0 (every shape here).
template <bool TRANSPOSE>
__device__ __forceinline__ void stage_matrix(_Float16* s, const _Float16* __restrict__ m, uint32_t rows, uint32_t cols,
                                             uint32_t rs, uint32_t zc, int tid, int nthr) {
	if (!TRANSPOSE) {
		if (cols % 8 == 0) {
			const uint32_t z8 = zc / 8, c8n = cols / 8;
			for (uint32_t idx = tid; idx < rows * z8; idx += nthr) {
				const uint32_t r = idx / z8, c8 = idx % z8;
				h8 v = h8{0, 0, 0, 0, 0, 0, 0, 0};
				if (c8 < c8n) v = *(const h8*)(m + (size_t)r * cols + 8 * c8);
				*(h8*)(s + r * rs + 8 * c8) = v;
			}
			return;
		}
		for (uint32_t idx = tid; idx < rows * zc; idx += nthr) {
			const uint32_t r = idx / zc, cc = idx % zc;
			s[r * rs + cc] = cc < cols ? m[r * cols + cc] : (_Float16)0.0f;
		}
	} else {
		// s[r][cc] = m[cc][r]: 16-byte loads along the rows of m, scattered into columns of s
		if (cols % 8 == 0) {
			const uint32_t c8n = cols / 8;
			for (uint32_t idx = tid; idx < rows * c8n; idx += nthr) {
				const uint32_t cc = idx / c8n, r0 = 8 * (idx % c8n);
				const h8 v = *(const h8*)(m + (size_t)cc * cols + r0);
#pragma unroll
				for (int e = 0; e < 8; ++e) s[(r0 + e) * rs + cc] = v[e];
			}
			for (uint32_t idx = tid; idx < cols * (zc - rows); idx += nthr) {
				const uint32_t r = idx / (zc - rows), cc = rows + idx % (zc - rows);
				s[r * rs + cc] = (_Float16)0.0f;
			}
			return;
		}
		for (uint32_t idx = tid; idx < zc * cols; idx += nthr) {
			const uint32_t cc = idx / cols, r = idx % cols;
			s[r * rs + cc] = cc < rows ? m[(size_t)cc * cols + r] : (_Float16)0.0f;
		}
	}
}

// B operand of one 32-sample slice: lane (c, q) of tile tau holds sample base + 16 tau + c,
// k = 32 s + 8 q .. +7 (16-byte loads; zero beyond K).
template <int KS>
__device__ __forceinline__ void load_slice_rows(h8 (&xb)[2][KS], const _Float16* __restrict__ in, uint32_t in_stride, uint32_t K,
                                                uint32_t base, int c, int q) {
#pragma unroll
	for (int tau = 0; tau < 2; ++tau) {
		const _Float16* row = in + (size_t)(base + 16 * tau + c) * in_stride;
#pragma unroll
		for (int s = 0; s < KS; ++s) {
			const uint32_t k0 = 32 * s + 8 * q;
			if (k0 < K) xb[tau][s] = *(const h8*)(row + k0);
			else xb[tau][s] = h8{0, 0, 0, 0, 0, 0, 0, 0};
		}
	}
}

// One 32-sample slice of  Out[i][16t + 4q + r] = epi( sum_k Amat[16t + c'][k] In[i][k] )  in the
// transposed MFMA form: A = LDS matrix rows (output features), B = the slice's input rows.
template <int NT, int KS, class Epi>
__device__ __forceinline__ void layer_slice_mma(const _Float16* sA, int rs, const h8 (&xb)[2][KS], int c, int q, Epi epi) {
	const f4 fz = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
	for (int t = 0; t < NT; ++t) {
		f4 a0 = fz, a1 = fz;
#pragma unroll
		for (int s = 0; s < KS; ++s) {
			const h8 af = *(const h8*)(sA + (16 * t + c) * rs + 32 * s + 8 * q);
			a0 = mfma16(af, xb[0][s], a0);
			a1 = mfma16(af, xb[1][s], a1);
		}
		epi(0, t, a0);
		epi(1, t, a1);
	}
}

// Persistent slice loop: the next slice's rows are in flight while this one multiplies.
template <int NT, int KS, class Epi, class Pre>
__device__ __forceinline__ void layer_slices(const _Float16* sA, int rs, const _Float16* __restrict__ in, uint32_t in_stride,
                                             uint32_t K, uint32_t B, int wave, int c, int q, Epi epi, Pre pre) {
	const uint32_t n_slices = B / 32, stride = gridDim.x * 4;
	uint32_t sl = blockIdx.x * 4 + wave;
	if (sl >= n_slices) return;
	h8 xb[2][KS];
	load_slice_rows<KS>(xb, in, in_stride, K, sl * 32, c, q);
	for (; sl < n_slices; sl += stride) {
		h8 xn[2][KS];
		const bool more = sl + stride < n_slices;
		if (more) load_slice_rows<KS>(xn, in, in_stride, K, (sl + stride) * 32, c, q);
		pre(sl * 32);  // epilogue operands of this slice, in flight during its MFMAs
		layer_slice_mma<NT, KS>(sA, rs, xb, c, q, [&](int tau, int t, f4 v) { epi(sl * 32, tau, t, v); });
		if (more) {
#pragma unroll
			for (int tau = 0; tau < 2; ++tau)
#pragma unroll
				for (int s = 0; s < KS; ++s) xb[tau][s] = xn[tau][s];
		}
	}
}


template <int A>  // ACT_NONE, ACT_RELU, or -1 (any, out of line)
__device__ __forceinline__ float act_fwd_sel(int a, float x) {
	if constexpr (A == ACT_NONE) return x;
	else if constexpr (A == ACT_RELU) return x > 0.0f ? x : 0.0f;
	else return act_fwd_ool(a, x);
}
template <int A>
__device__ __forceinline__ float act_bwd_sel(int a, float g, float y) {
	if constexpr (A == ACT_NONE) return g;
	else if constexpr (A == ACT_RELU) return y > 0.0f ? g : 0.0f;
	else return act_bwd_ool(a, g, y);
}

// run f with the activation as a compile-time constant where it is None / ReLU
template <class F>
__device__ __forceinline__ void with_act(int act, F f) {
	if (act == ACT_NONE) f(std::integral_constant<int, ACT_NONE>{});
	else if (act == ACT_RELU) f(std::integral_constant<int, ACT_RELU>{});
	else f(std::integral_constant<int, -1>{});
}

template <int NT, int KS>
__global__ __launch_bounds__(256, 2) void k_layer_fwd(uint32_t B, uint32_t K, const _Float16* __restrict__ w,
                                                    const _Float16* __restrict__ x, _Float16* __restrict__ y, int act) {
	constexpr int N = 16 * NT, RS = 32 * KS + 8;
	__shared__ __attribute__((aligned(16))) _Float16 sW[N * RS];
	const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	const int c = lane & 15, q = lane >> 4;
	stage_matrix<false>(sW, w, N, K, RS, 32 * KS, tid, 256);
	__syncthreads();
	with_act(act, [&](auto A) {
		layer_slices<NT, KS>(sW, RS, x, K, K, B, wave, c, q, [&](uint32_t base, int tau, int t, f4 v) {
			h4 o;
#pragma unroll
			for (int r = 0; r < 4; ++r) o[r] = f16_rn(act_fwd_sel<decltype(A)::value>(act, v[r]));
			*(h4*)(y + (size_t)(base + 16 * tau + c) * N + 16 * t + 4 * q) = o;
		}, [](uint32_t) {});
	});
}

// dX[i][k] = act'(H[i][k]) * sum_n dY[i][n] W[n][k]; H == nullptr -> no transfer. K = 16 NT.
template <int NT, int KS>
__global__ __launch_bounds__(256, 2) void k_layer_bwd(uint32_t B, uint32_t N, const _Float16* __restrict__ w,
                                                    const _Float16* __restrict__ dy, const _Float16* __restrict__ h,
                                                    _Float16* __restrict__ dx, int act, uint32_t pairs) {
	constexpr int K = 16 * NT, RS = 32 * KS + 8;
	__shared__ __attribute__((aligned(16))) _Float16 sWT[K * RS];
	const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	const int c = lane & 15, q = lane >> 4;
	stage_matrix<true>(sWT, w, N, K, RS, 32 * KS, tid, 256);
	__syncthreads();
	with_act(h ? act : ACT_NONE, [&](auto A) {
		constexpr bool TRANSFER = decltype(A)::value != ACT_NONE;
		h4 hv[2][NT];
		layer_slices<NT, KS>(sWT, RS, dy, N, N, B, wave, c, q, [&](uint32_t base, int tau, int t, f4 v) {
			const size_t o = (size_t)(base + 16 * tau + c) * K + 16 * t + 4 * q;
			h4 r4;
			if constexpr (TRANSFER) {
#pragma unroll
				for (int r = 0; r < 4; ++r) r4[r] = f16_rn(act_bwd_sel<decltype(A)::value>(act, v[r], (float)hv[tau][t][r]));
			} else {
#pragma unroll
				for (int r = 0; r < 4; ++r) r4[r] = (_Float16)v[r];
				if (pairs) {  // grid dL/d(encoding) as level-major feature pairs [K/2][B] (the fused kernel's layout)
					const uint32_t lv = 8 * t + 2 * q, i = base + 16 * tau + c;
					uint32_t* d2 = (uint32_t*)dx;
					d2[(size_t)lv * B + i] = __builtin_bit_cast(uint32_t, h2{r4[0], r4[1]});
					d2[(size_t)(lv + 1) * B + i] = __builtin_bit_cast(uint32_t, h2{r4[2], r4[3]});
					return;
				}
			}
			*(h4*)(dx + o) = r4;
		}, [&](uint32_t base) {
			if constexpr (TRANSFER) {
#pragma unroll
				for (int tau = 0; tau < 2; ++tau)
#pragma unroll
					for (int t = 0; t < NT; ++t) hv[tau][t] = *(const h4*)(h + (size_t)(base + 16 * tau + c) * K + 16 * t + 4 * q);
			}
		});
	});
}

// Weight-gradient partial of one sample chunk: P[n][k] = sum_{i in chunk} dY[i][n] X[i][k].
// 8 waves stage 64 samples of dY and X per step in LDS (double-buffered: the next step's rows are
// loaded into registers before this step's MFMAs and written to the other buffer after them, so
// the HBM latency overlaps the math); wave w owns output tiles w, w+8, ... (MT x KT tiles of
// 16x16) with fp32 accumulators for the whole chunk.
constexpr int WG_WAVES = 8, WG_STEP = 64;
// Widths above 128 (wgrad_blocks): blockIdx.y / blockIdx.z pick the output block [n0, n0 + 16 MT) x
// [k0, k0 + 16 KT) of a dW of ldp = ldx columns; dy rows have ldd halves, x rows ldx.
template <int MT, int KT>
__global__ __launch_bounds__(WG_WAVES * 64) void k_wgrad(uint32_t B, uint32_t pts_per_chunk, const _Float16* __restrict__ dy,
                                                         const _Float16* __restrict__ x, float* __restrict__ partial, uint32_t ldd,
                                                         uint32_t ldx, uint32_t n_rows, uint32_t nb0, uint32_t kb0) {
	constexpr int N = 16 * MT, K = 16 * KT, RSD = N + 8, RSX = K + 8, NTHR = WG_WAVES * 64;
	const uint32_t n0 = nb0 + blockIdx.y * N, k0 = kb0 + blockIdx.z * K;
	dy += n0;
	x += k0;
	constexpr int TILES = MT * KT, TPW = (TILES + WG_WAVES - 1) / WG_WAVES;
	constexpr int VD = WG_STEP * N / 8, VX = WG_STEP * K / 8;  // 16-byte vectors per step
	constexpr int PD = (VD + NTHR - 1) / NTHR, PX = (VX + NTHR - 1) / NTHR;
	__shared__ __attribute__((aligned(16))) _Float16 sD[2][WG_STEP * RSD];
	__shared__ __attribute__((aligned(16))) _Float16 sX[2][WG_STEP * RSX];
	const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	const int c = lane & 15, q = lane >> 4;
	const f4 fz = {0.0f, 0.0f, 0.0f, 0.0f};
	f4 acc[TPW];
#pragma unroll
	for (int m = 0; m < TPW; ++m) acc[m] = fz;
	const uint32_t i0 = blockIdx.x * pts_per_chunk;
	const uint32_t i1 = min(B, i0 + pts_per_chunk);
	h8 rd[PD], rx[PX];
	auto load = [&](uint32_t b0) {
#pragma unroll
		for (int j = 0; j < PD; ++j) {
			const int idx = tid + j * NTHR;
			const int r = idx / (N / 8), c8 = idx % (N / 8);
			rd[j] = (idx < VD && b0 + r < i1) ? *(const h8*)(dy + (size_t)(b0 + r) * ldd + 8 * c8) : h8{0, 0, 0, 0, 0, 0, 0, 0};
		}
#pragma unroll
		for (int j = 0; j < PX; ++j) {
			const int idx = tid + j * NTHR;
			const int r = idx / (K / 8), c8 = idx % (K / 8);
			rx[j] = (idx < VX && b0 + r < i1) ? *(const h8*)(x + (size_t)(b0 + r) * ldx + 8 * c8) : h8{0, 0, 0, 0, 0, 0, 0, 0};
		}
	};
	auto store = [&](int buf) {
#pragma unroll
		for (int j = 0; j < PD; ++j) {
			const int idx = tid + j * NTHR;
			if (idx < VD) *(h8*)(&sD[buf][(idx / (N / 8)) * RSD + 8 * (idx % (N / 8))]) = rd[j];
		}
#pragma unroll
		for (int j = 0; j < PX; ++j) {
			const int idx = tid + j * NTHR;
			if (idx < VX) *(h8*)(&sX[buf][(idx / (K / 8)) * RSX + 8 * (idx % (K / 8))]) = rx[j];
		}
	};
	int buf = 0;
	if (i0 < i1) {
		load(i0);
		store(0);
	}
	__syncthreads();
	for (uint32_t b0 = i0; b0 < i1; b0 += WG_STEP) {
		const bool more = b0 + WG_STEP < i1;
		if (more) load(b0 + WG_STEP);
#pragma unroll
		for (int h = 0; h < WG_STEP / 32; ++h) {
			const _Float16* dD = sD[buf] + 32 * h * RSD;
			const _Float16* dX = sX[buf] + 32 * h * RSX;
#pragma unroll
			for (int m = 0; m < TPW; ++m) {
				const int j = wave + WG_WAVES * m;
				if (j < TILES) {
					const int mt = j / KT, kt = j % KT;
					acc[m] = mfma16(lds_trfrag(dD, RSD, q, c, mt), lds_trfrag(dX, RSX, q, c, kt), acc[m]);
				}
			}
		}
		if (more) store(buf ^ 1);
		__syncthreads();
		buf ^= 1;
	}
	float* dst = partial + (size_t)blockIdx.x * n_rows * ldx + (size_t)n0 * ldx + k0;
#pragma unroll
	for (int m = 0; m < TPW; ++m) {
		const int j = wave + WG_WAVES * m;
		if (j < TILES) {
			const int mt = j / KT, kt = j % KT;
#pragma unroll
			for (int r = 0; r < 4; ++r) dst[(size_t)(16 * mt + 4 * q + r) * ldx + 16 * kt + c] = acc[m][r];
		}
	}
}

// Layers wider than the register kernels above (CutlassMLP widths above 128, encodings wider than 128,
// padded outputs above 128; reference cutlass_mlp.cu:41-81, fully_fused_mlp.cu:591): one output block
// of 16 NT features per blockIdx.y, its A rows staged once in dynamic LDS over the whole contraction
// C (zero-filled to a multiple of 32), persistent 32-sample slices per wave with the contraction as a
// runtime loop (the next 32-wide step's input rows in flight during this step's MFMAs).
//   TR = false (forward):  Out[i][o] = act( sum_c W[o][c] In[i][c] ),         W [n_out][C]
//   TR = true  (backward): Out[i][o] = act'(H[i][o]) * sum_c W[c][o] In[i][c], W [C][n_out]
template <int NT, bool TR>
__global__ __launch_bounds__(256, 1) void k_wide_layer(uint32_t B, uint32_t C, uint32_t n_out, const _Float16* __restrict__ w,
                                                     const _Float16* __restrict__ in, _Float16* __restrict__ out,
                                                     const _Float16* __restrict__ h, int act, uint32_t pairs) {
	extern __shared__ __attribute__((aligned(16))) _Float16 sA[];
	const uint32_t Cp = (C + 31) / 32 * 32, rs = Cp + 8;
	const uint32_t o0 = blockIdx.y * 16 * NT;
	const uint32_t ntv = min((uint32_t)NT, (n_out - o0) / 16);  // valid 16-row tiles of this block
	const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	const int c = lane & 15, q = lane >> 4;
	// stage A = rows o0 .. o0 + 16 NT of W (TR: of W^T), zero outside [n_out) x [C)
	if (!TR) {
		const uint32_t c8n = Cp / 8;
		for (uint32_t idx = tid; idx < 16u * NT * c8n; idx += 256) {
			const uint32_t r = idx / c8n, c8 = idx % c8n;
			h8 v = h8{0, 0, 0, 0, 0, 0, 0, 0};
			if (o0 + r < n_out && 8 * c8 < C) v = *(const h8*)(w + (size_t)(o0 + r) * C + 8 * c8);
			*(h8*)(sA + r * rs + 8 * c8) = v;
		}
	} else {
		constexpr uint32_t R8 = 2 * NT;  // 8-wide row groups of the block
		for (uint32_t idx = tid; idx < Cp * R8; idx += 256) {
			const uint32_t cc = idx / R8, r0 = 8 * (idx % R8);
			h8 v = h8{0, 0, 0, 0, 0, 0, 0, 0};
			if (cc < C && o0 + r0 < n_out) v = *(const h8*)(w + (size_t)cc * n_out + o0 + r0);
#pragma unroll
			for (int e = 0; e < 8; ++e) sA[(r0 + e) * rs + cc] = v[e];
		}
	}
	__syncthreads();
	const uint32_t n_slices = B / 32, stride = gridDim.x * 4;
	const f4 fz = {0.0f, 0.0f, 0.0f, 0.0f};
	const uint32_t steps = Cp / 32;
	auto load = [&](h8 (&xb)[2], uint32_t base, uint32_t s) {
#pragma unroll
		for (int tau = 0; tau < 2; ++tau) {
			const uint32_t k = 32 * s + 8 * q;
			xb[tau] = k < C ? *(const h8*)(in + (size_t)(base + 16 * tau + c) * C + k) : h8{0, 0, 0, 0, 0, 0, 0, 0};
		}
	};
	with_act(act, [&](auto A) {
		constexpr int AC = decltype(A)::value;
		for (uint32_t sl = blockIdx.x * 4 + wave; sl < n_slices; sl += stride) {
			const uint32_t base = sl * 32;
			f4 acc[NT][2];
#pragma unroll
			for (int t = 0; t < NT; ++t) acc[t][0] = acc[t][1] = fz;
			h8 xb[2], xn[2];
			load(xb, base, 0);
			for (uint32_t s = 0; s < steps; ++s) {
				if (s + 1 < steps) load(xn, base, s + 1);
#pragma unroll
				for (int t = 0; t < NT; ++t) {
					if ((uint32_t)t < ntv) {
						const h8 af = *(const h8*)(sA + (16 * t + c) * rs + 32 * s + 8 * q);
						acc[t][0] = mfma16(af, xb[0], acc[t][0]);
						acc[t][1] = mfma16(af, xb[1], acc[t][1]);
					}
				}
				xb[0] = xn[0];
				xb[1] = xn[1];
			}
#pragma unroll
			for (int t = 0; t < NT; ++t) {
				if ((uint32_t)t >= ntv) continue;
#pragma unroll
				for (int tau = 0; tau < 2; ++tau) {
					const uint32_t i = base + 16 * tau + c, o = o0 + 16 * t + 4 * q;
					const f4 v = acc[t][tau];
					h4 r4;
					if constexpr (!TR) {
#pragma unroll
						for (int r = 0; r < 4; ++r) r4[r] = f16_rn(act_fwd_sel<AC>(act, v[r]));
					} else if constexpr (AC != ACT_NONE) {
						const h4 hv = *(const h4*)(h + (size_t)i * n_out + o);
#pragma unroll
						for (int r = 0; r < 4; ++r) r4[r] = f16_rn(act_bwd_sel<AC>(act, v[r], (float)hv[r]));
					} else {
#pragma unroll
						for (int r = 0; r < 4; ++r) r4[r] = (_Float16)v[r];
						if (pairs) {  // level-major feature pairs [n_out / 2][B] (grid F = 2)
							uint32_t* d2 = (uint32_t*)out;
							d2[(size_t)(o / 2) * B + i] = __builtin_bit_cast(uint32_t, h2{r4[0], r4[1]});
							d2[(size_t)(o / 2 + 1) * B + i] = __builtin_bit_cast(uint32_t, h2{r4[2], r4[3]});
							continue;
						}
					}
					*(h4*)(out + (size_t)i * n_out + o) = r4;
				}
			}
		}
	});
}

// NT (output rows per block / 16) of the wide kernel: the staged rows of the whole contraction must fit
// 160 KB of LDS: 128 rows up to C = 512, 64 up to 1024, 32 up to 2048, 16 up to 4096
static uint32_t wide_nt(uint32_t C) {
	const uint32_t rs = (C + 31) / 32 * 32 + 8;
	for (uint32_t nt = 8; nt >= 1; nt /= 2)
		if (16 * nt * rs * 2 <= 160 * 1024) return nt;
	return 0;
}

static void launch_wide_layer(hipStream_t st, bool tr, uint32_t B, uint32_t C, uint32_t n_out, const void* w16, const void* in16, void* out16,
                              const void* h16, int act, bool pairs) {
	const uint32_t nt = wide_nt(C);
	TCNN_CHECK(nt > 0, "layer: contraction width " + std::to_string(C) + " exceeds the wide layer kernel's LDS (4096)");
	const uint32_t ny = div_round_up(n_out, 16 * nt);
	const uint32_t gx = std::max(1u, std::min(div_round_up(B / 32, 4), std::max(1u, 512u / ny)));
	const size_t lds = (size_t)16 * nt * ((C + 31) / 32 * 32 + 8) * 2;
	const dim3 g(gx, ny);
#define WIDE(NT_, TR_)                                                                                                         \
	{                                                                                                                         \
		static uint64_t done = 0;                                                                                             \
		set_dyn_lds((const void*)k_wide_layer<NT_, TR_>, 160 * 1024, done);                                                   \
		hipLaunchKernelGGL((k_wide_layer<NT_, TR_>), g, dim3(256), lds, st, B, C, n_out, (const _Float16*)w16, (const _Float16*)in16, \
		                   (_Float16*)out16, (const _Float16*)h16, act, pairs ? 1u : 0u);                                    \
	}
	if (tr) {
		switch (nt) { case 8: WIDE(8, true) break; case 4: WIDE(4, true) break; case 2: WIDE(2, true) break; default: WIDE(1, true) }
	} else {
		switch (nt) { case 8: WIDE(8, false) break; case 4: WIDE(4, false) break; case 2: WIDE(2, false) break; default: WIDE(1, false) }
	}
#undef WIDE
	TCNN_HIP_CHECK(hipGetLastError());
}

// ---- launchers ----
static uint32_t pow2_ceil_steps(uint32_t k) {  // 32-wide K steps, rounded up to 1, 2, 4 (K <= 128)
	const uint32_t s = div_round_up(k, 32);
	return s <= 1 ? 1 : s <= 2 ? 2 : s <= 4 ? 4 : 0;
}

// persistent: two workgroups per CU (the weights are staged once per workgroup)
static uint32_t layer_blocks(uint32_t B) { return std::max(1u, std::min(div_round_up(B / 32, 4), 512u)); }

// CutlassMLP widths (reference cutlass_mlp.h:115-121, REQUIRED_ALIGNMENT 16): any multiple of 16 --
// up to 128 on the register-tiled layer kernels (output tiles 1..8; K zero-filled to 32, 64 or 128),
// above that (or a contraction above 128) on k_wide_layer, contractions up to 4096.
bool layered_width_supported(uint32_t w) { return w >= 16 && w <= 4096 && w % 16 == 0; }

#define TCNN_KS_DISPATCH(NT_, KSV, CALL)                                                                  \
	switch (KSV) { case 1: CALL(NT_, 1); break; case 2: CALL(NT_, 2); break; case 4: CALL(NT_, 4); break; default: ok = false; }
#define TCNN_LAYER_DISPATCH(NTV, KSV, CALL)                                                              \
	switch (NTV) {                                                                                       \
		case 1: TCNN_KS_DISPATCH(1, KSV, CALL) break; case 2: TCNN_KS_DISPATCH(2, KSV, CALL) break;      \
		case 3: TCNN_KS_DISPATCH(3, KSV, CALL) break; case 4: TCNN_KS_DISPATCH(4, KSV, CALL) break;      \
		case 5: TCNN_KS_DISPATCH(5, KSV, CALL) break; case 6: TCNN_KS_DISPATCH(6, KSV, CALL) break;      \
		case 7: TCNN_KS_DISPATCH(7, KSV, CALL) break; case 8: TCNN_KS_DISPATCH(8, KSV, CALL) break;      \
		default: ok = false;                                                                             \
	}

void launch_layer_fwd(hipStream_t st, uint32_t B, uint32_t N, uint32_t K, const void* w16, const void* x16, void* y16, int act) {
	TCNN_CHECK(B % 32 == 0 && N % 16 == 0 && K % 16 == 0, "layer_fwd: B % 32, N % 16, K % 16 must be 0");
	if (B == 0) return;
	if (N > 128 || K > 128) {
		launch_wide_layer(st, false, B, K, N, w16, x16, y16, nullptr, act, false);
		return;
	}
	bool ok = true;
	const dim3 g(layer_blocks(B));
#define CALL(nt, ks) hipLaunchKernelGGL((k_layer_fwd<nt, ks>), g, dim3(256), 0, st, B, K, (const _Float16*)w16, (const _Float16*)x16, (_Float16*)y16, act)
	TCNN_LAYER_DISPATCH(N / 16, pow2_ceil_steps(K), CALL)
#undef CALL
	TCNN_CHECK(ok, "layer_fwd: unsupported shape N=" + std::to_string(N) + " K=" + std::to_string(K));
	TCNN_HIP_CHECK(hipGetLastError());
}

void launch_layer_bwd(hipStream_t st, uint32_t B, uint32_t N, uint32_t K, const void* w16, const void* dy16, const void* h16,
                      void* dx16, int act, bool pairs) {
	TCNN_CHECK(!pairs || !h16, "layer_bwd: the pairs layout is for the untransferred encoding gradient");
	TCNN_CHECK(B % 32 == 0 && N % 16 == 0 && K % 16 == 0, "layer_bwd: B % 32, N % 16, K % 16 must be 0");
	if (B == 0) return;
	if (N > 128 || K > 128) {
		launch_wide_layer(st, true, B, N, K, w16, dy16, dx16, h16, h16 ? act : ACT_NONE, pairs);
		return;
	}
	bool ok = true;
	const dim3 g(layer_blocks(B));
#define CALL(nt, ks) hipLaunchKernelGGL((k_layer_bwd<nt, ks>), g, dim3(256), 0, st, B, N, (const _Float16*)w16, (const _Float16*)dy16, (const _Float16*)h16, (_Float16*)dx16, act, pairs ? 1u : 0u)
	TCNN_LAYER_DISPATCH(K / 16, pow2_ceil_steps(N), CALL)
#undef CALL
	TCNN_CHECK(ok, "layer_bwd: unsupported shape N=" + std::to_string(N) + " K=" + std::to_string(K));
	TCNN_HIP_CHECK(hipGetLastError());
}

uint32_t wgrad_n_chunks(uint32_t B) { return std::max(1u, std::min(B / 1024u, 256u)); }

void launch_wgrad(hipStream_t st, uint32_t B, uint32_t N, uint32_t K, const void* dy16, const void* x16, float* partial,
                  uint32_t n_chunks) {
	TCNN_CHECK(B % 32 == 0 && N % 16 == 0 && K % 16 == 0, "wgrad: B % 32, N % 16, K % 16 must be 0");
	if (B == 0) return;
	const uint32_t ppc = div_round_up(div_round_up(B, n_chunks), 32) * 32;
	const uint32_t nc = div_round_up(B, ppc);
	TCNN_CHECK(nc <= n_chunks, "wgrad: chunk plan");
	if (nc < n_chunks) TCNN_HIP_CHECK(hipMemsetAsync(partial + (size_t)nc * N * K, 0, (size_t)(n_chunks - nc) * N * K * 4, st));
	bool ok = true;
	// blocks of up to 128 x 128 outputs: the full blocks in one launch, the remainder rows / columns
	// (N % 128, K % 128: 16 .. 112) in up to three more; MT, KT = tiles of 16 per block (1..8)
	const uint32_t nfull = N / 128, kfull = K / 128, nrem = (N % 128) / 16, krem = (K % 128) / 16;
	auto one = [&](uint32_t mt, uint32_t kt, uint32_t gy, uint32_t gz, uint32_t nb0, uint32_t kb0) {
		if (!mt || !kt || !gy || !gz) return;
		const dim3 g(nc, gy, gz);
#define WG(m_, k_) hipLaunchKernelGGL((k_wgrad<m_, k_>), g, dim3(WG_WAVES * 64), 0, st, B, ppc, (const _Float16*)dy16, (const _Float16*)x16, partial, N, K, N, nb0, kb0)
#define WGK(m_)                                                                          \
		switch (kt) {                                                                    \
			case 1: WG(m_, 1); break; case 2: WG(m_, 2); break; case 3: WG(m_, 3); break;    \
			case 4: WG(m_, 4); break; case 5: WG(m_, 5); break; case 6: WG(m_, 6); break;    \
			case 7: WG(m_, 7); break; case 8: WG(m_, 8); break; default: ok = false;         \
		}
		switch (mt) {
			case 1: WGK(1); break; case 2: WGK(2); break; case 3: WGK(3); break; case 4: WGK(4); break;
			case 5: WGK(5); break; case 6: WGK(6); break; case 7: WGK(7); break; case 8: WGK(8); break;
			default: ok = false;
		}
#undef WGK
#undef WG
	};
	if (N <= 128 && K <= 128) {
		one(N / 16, K / 16, 1, 1, 0, 0);  // the common case: one block
	} else {
		one(8, 8, nfull, kfull, 0, 0);
		one(8, krem, nfull, 1, 0, 128 * kfull);
		one(nrem, 8, 1, kfull, 128 * nfull, 0);
		one(nrem, krem, 1, 1, 128 * nfull, 128 * kfull);
	}
	TCNN_CHECK(ok, "wgrad: unsupported shape N=" + std::to_string(N) + " K=" + std::to_string(K));
	TCNN_HIP_CHECK(hipGetLastError());
}

// RelativeL2 (losses/relative_l2.h:40-76) or L2 (losses/l2.h:40-76, l2 != 0) over pred fp16
// [B][stride]; per-workgroup loss sums.
__global__ __launch_bounds__(256) void k_relative_l2_partial(uint32_t l2, uint32_t n_elements, uint32_t stride, uint32_t dims, float loss_scale,
                                                              float n_total, const _Float16* __restrict__ pred,
                                                              const float* __restrict__ target, _Float16* __restrict__ grads,
                                                              float* __restrict__ loss_partial, const float* __restrict__ pdf) {
	__shared__ float part[4];
	float s = 0.0f;
	for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n_elements; i += gridDim.x * 256) {
		const uint32_t intra = i % stride, inter = i / stride;
		if (intra >= dims) {
			grads[i] = (_Float16)0.0f;
			continue;
		}
		const float p = (float)pred[i];
		const float pse = l2 ? 1.0f : __builtin_fmaf(p, p, 0.01f);
		const float d = p - target[inter * dims + intra];
		if (pdf) {  // data_pdf (relative_l2.h:64-72, l2.h:63-71): values and gradient divided by the pdf
			const float f = pdf[inter * dims + intra];
			s += d * d / pse / f / n_total;
			grads[i] = f16_rn(loss_scale * (2.0f * d / pse / f) / n_total);
			continue;
		}
		s += d * d / pse / n_total;
		const float gr = 2.0f * d / pse;
		grads[i] = f16_rn(loss_scale * gr / n_total);
	}
#pragma unroll
	for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
	if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
	__syncthreads();
	if (threadIdx.x == 0) loss_partial[blockIdx.x] = (part[0] + part[1]) + (part[2] + part[3]);
}

uint32_t relative_l2_n_blocks(uint32_t B, uint32_t stride) { return std::max(1u, std::min(div_round_up((uint64_t)B * stride, 256), 1024u)); }

void launch_relative_l2_partial(hipStream_t st, uint32_t B, uint32_t stride, uint32_t dims, float loss_scale, const void* pred16,
                                const float* target, void* grads16, float* loss_partial, uint32_t loss_l2, const float* pdf) {
	const uint32_t n = B * stride;
	if (!n) return;
	hipLaunchKernelGGL(k_relative_l2_partial, dim3(relative_l2_n_blocks(B, stride)), dim3(256), 0, st, loss_l2, n, stride, dims, loss_scale,
	                   (float)((uint64_t)B * dims), (const _Float16*)pred16, target, (_Float16*)grads16, loss_partial, pdf);
	TCNN_HIP_CHECK(hipGetLastError());
}

__global__ __launch_bounds__(256) void k_act_bwd_inplace(uint32_t n, int act, const _Float16* __restrict__ y, _Float16* __restrict__ g) {
	const uint32_t i = blockIdx.x * 256 + threadIdx.x;
	if (i < n) g[i] = f16_rn(act_bwd_rt(act, (float)g[i], (float)y[i]));
}

void launch_act_bwd_inplace(hipStream_t st, uint32_t n, int act, const void* y16, void* g16) {
	if (!n || act == ACT_NONE) return;
	hipLaunchKernelGGL(k_act_bwd_inplace, dim3(div_round_up(n, 256)), dim3(256), 0, st, n, act, (const _Float16*)y16, (_Float16*)g16);
	TCNN_HIP_CHECK(hipGetLastError());
}

}  // namespace tcnn_amd
