// mlp_fused.h -- fully fused MLP engine for gfx950 (MFMA f32_16x16x32_f16, wave64).
//
// What the reference does (src/fully_fused_mlp.cu): one WMMA kernel per direction with fp16
// accumulators, hidden activations round-tripped through HBM, and CUTLASS split-K GEMMs for the
// weight gradients (fully_fused_mlp.cu:735-836). This engine instead keeps every activation of a
// 32-sample slice in registers for the whole forward + loss + backward + weight-gradient pass:
//
//   * "transposed" formulation: each layer computes Y^T[neuron][sample] = W[neuron][k] X^T[k][sample]
//     so the MFMA accumulator (D: lane = sample, 4 consecutive neurons per lane) is directly the next
//     layer's B operand (k = neuron) after an f32->f16 pack, with the k order permuted inside each
//     32-wide k step:  k_s(8q+e) = 32s + 16(e>>2) + 4q + (e&3)   (q = lane>>4).
//     The A operands (weights, W and W^T) are read from LDS with the same permutation.
//   * weight gradients contract over samples, so the slice's activations / deltas are staged
//     through a per-wave LDS buffer laid out [sample][neuron] and read back with the gfx950
//     ds_read_b64_tr_b16 transpose read; dW accumulates in registers across all slices a wave
//     processes and is reduced once per workgroup into an fp32 partial slab.
//   * the grid encoding (when the input is a hash grid) is computed in-register in exactly the
//     B-fragment order, and dL/d(encoding) leaves the kernel in the level-major half2 layout the
//     grid backward kernel consumes.
// fp16 storage points are the reference's (activations, output, dL/dy, backprop temporaries);
// accumulation is fp32 (MFMA).
#pragma once

#include "common.h"
#include "grid_device.h"

namespace tcnn_amd {

enum class Act : int { None = 0, ReLU = 1 };

__device__ __forceinline__ f4 mfma16(h8 a, h8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

__device__ __forceinline__ h8 cat8(h4 lo, h4 hi) { return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7); }

__device__ __forceinline__ h4 zero4() { return h4{(_Float16)0.0f, (_Float16)0.0f, (_Float16)0.0f, (_Float16)0.0f}; }

template <Act A>
__device__ __forceinline__ h4 act_fwd(f4 v) {
	if constexpr (A == Act::ReLU) {
		v[0] = v[0] > 0.0f ? v[0] : 0.0f; v[1] = v[1] > 0.0f ? v[1] : 0.0f;
		v[2] = v[2] > 0.0f ? v[2] : 0.0f; v[3] = v[3] > 0.0f ? v[3] : 0.0f;
	}
	return __builtin_convertvector(v, h4);
}

// activation transfer given the post-activation value (reference common_device.h:240-297)
template <Act A>
__device__ __forceinline__ h4 act_bwd(h4 fwd, f4 g) {
	h4 r = __builtin_convertvector(g, h4);
	if constexpr (A == Act::ReLU) {
#pragma unroll
		for (int k = 0; k < 4; ++k) r[k] = fwd[k] > (_Float16)0.0f ? r[k] : (_Float16)0.0f;
	}
	return r;
}

// A operand from a row-major LDS matrix M[row][col] (row stride rs halves):
// lane (c, q) takes M[row][col0 + 0..3] and M[row][col0 + 16 + 0..3], col0 = 32s + 4q.
__device__ __forceinline__ h8 lds_afrag(const _Float16* M, int rs, int row, int col0) {
	const h4 lo = *(const h4*)(M + row * rs + col0);
	const h4 hi = *(const h4*)(M + row * rs + col0 + 16);
	return cat8(lo, hi);
}

// Operand with samples along K from a staging buffer S[32 samples][rs]: lane (c, q) receives
// S[8q + e][16*tile + c], e = 0..7, via two ds_read_b64_tr_b16 (CDNA4 transpose read).
__device__ __forceinline__ h8 lds_trfrag(const _Float16* S, int rs, int q, int c, int tile) {
	const int row = 8 * q + (c >> 2);
	const int col = 16 * tile + 4 * (c & 3);
	typedef __attribute__((address_space(3))) s4 lds_s4;
	const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(S + row * rs + col));
	const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(S + (row + 4) * rs + col));
	return cat8(__builtin_bit_cast(h4, lo), __builtin_bit_cast(h4, hi));
}

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <int W, int IN, int NH>
struct FusedLayout {
	static_assert(W % 32 == 0 && IN % 32 == 0 && NH >= 1, "fused MLP: W, IN multiples of 32");
	static constexpr int NT = W / 16, KW = W / 32, NTI = IN / 16, KI = IN / 32;
	static constexpr int NHM = NH - 1;  // hidden WxW matrices
	static constexpr int RSI = IN + 8, RSW = W + 8, RSO = 24;
	static constexpr int RSS = (W > IN ? W : IN) + 8;
	static constexpr int oW0 = 0;
	static constexpr int oW0T = oW0 + W * RSI;
	static constexpr int oWh = oW0T + IN * RSW;
	static constexpr int oWhT = oWh + NHM * W * RSW;
	static constexpr int oWo = oWhT + NHM * W * RSW;
	static constexpr int oWoT = oWo + 16 * RSW;
	static constexpr int oStage = oWoT + W * RSO;
	static constexpr int STAGE = 32 * RSS;  // one [32][RSS] buffer
	static constexpr int WAVES = 4;
	static constexpr int oEnd = oStage + WAVES * 2 * STAGE;
	static constexpr int LVL_BYTES = oEnd * 2;          // LevelInfo table (byte offset)
	static constexpr int N_MLP = W * IN + NHM * W * W + 16 * W;
	static constexpr int BYTES_MAIN = LVL_BYTES + (int)MAX_LEVELS * 16;
	static constexpr int BYTES_RED = (N_MLP + 4) * 4;
	static constexpr int BYTES = BYTES_MAIN > BYTES_RED ? BYTES_MAIN : BYTES_RED;
	static_assert(oW0T % 8 == 0 && oWh % 8 == 0 && oWhT % 8 == 0 && oWo % 8 == 0 && oWoT % 8 == 0 && oStage % 8 == 0, "16B alignment");
};

// Cooperative copy of the fp16 weights into LDS, row-major and transposed, padded rows.
template <int W, int IN, int NH>
__device__ __forceinline__ void load_weights_lds(_Float16* smem, const _Float16* __restrict__ params, int tid, int nthreads) {
	using L = FusedLayout<W, IN, NH>;
	const uint16_t* p = (const uint16_t*)params;
	uint16_t* s = (uint16_t*)smem;
	for (int idx = tid; idx < W * IN; idx += nthreads) {
		const int n = idx / IN, k = idx % IN;
		const uint16_t v = p[idx];
		s[L::oW0 + n * L::RSI + k] = v;
		s[L::oW0T + k * L::RSW + n] = v;
	}
	p += W * IN;
	for (int j = 0; j < L::NHM; ++j) {
		for (int idx = tid; idx < W * W; idx += nthreads) {
			const int n = idx / W, k = idx % W;
			const uint16_t v = p[idx];
			s[L::oWh + j * W * L::RSW + n * L::RSW + k] = v;
			s[L::oWhT + j * W * L::RSW + k * L::RSW + n] = v;
		}
		p += W * W;
	}
	for (int idx = tid; idx < 16 * W; idx += nthreads) {
		const int o = idx / W, k = idx % W;
		const uint16_t v = p[idx];
		s[L::oWo + o * L::RSW + k] = v;
		s[L::oWoT + k * L::RSO + o] = v;
	}
}

// The LDS weight image (W, W^T, padded rows) is built once per step by k_pack_weights into global
// memory; every workgroup then copies it with 16-byte loads instead of re-transposing the weights.
template <int W, int IN, int NH>
__global__ void k_pack_weights(const _Float16* __restrict__ params, _Float16* __restrict__ image) {
	load_weights_lds<W, IN, NH>(image, params, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
}

__device__ __forceinline__ void copy_image_to_lds(_Float16* smem, const _Float16* __restrict__ image, int n_halves, int tid, int nthreads) {
	const uint4* src = (const uint4*)image;
	uint4* dst = (uint4*)smem;
	const int n16 = n_halves / 8;
	for (int k = tid; k < n16; k += nthreads) dst[k] = src[k];
}

struct FusedTrainArgs {
	const _Float16* wimage; // packed LDS weight image (k_pack_weights)
	uint32_t B;
	uint32_t dims;          // target width (n_output_dims)
	float loss_scale;
	float n_total;          // (float)(B * dims) as in relative_l2.h:64
	const _Float16* params; // MLP weights fp16 [W0 | hidden | Wout]
	const uint32_t* table;  // grid params as half2 entries (F == 2)
	const float* pos;       // [B][D]
	const float* target;    // [B][dims]
	_Float16* out;          // optional network output [B][16]
	uint32_t* dLdenc;       // [L][B] half2 (level-major feature pairs)
	float* wgrad_partial;   // [gridDim.x][N_MLP]
	float* loss_partial;    // [gridDim.x]
	const LevelInfo* levels;
	uint32_t hash_grid;
	uint32_t interp;
	const _Float16* dout;   // EXT_DOUT: external dL/d(output) fp16 [B][16] (loss-scaled by the caller)
};

// One workgroup = 4 waves; each wave processes 32-sample slices in a grid-stride loop.
template <int W, int IN, int NH, uint32_t D, HashType H, Act ACT, bool EXT_DOUT>
__global__ __launch_bounds__(256, 2) void k_fused_train_grid(const FusedTrainArgs a) {
	using L = FusedLayout<W, IN, NH>;
	constexpr int NT = L::NT, KW = L::KW, NTI = L::NTI, KI = L::KI, NHM = L::NHM;
	constexpr int NLVL = IN / 2;
	extern __shared__ __attribute__((aligned(16))) _Float16 smem[];

	const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	const int c = lane & 15, q = lane >> 4;

	copy_image_to_lds(smem, a.wimage, L::oStage, tid, 256);
	LevelInfo* sLvl = (LevelInfo*)((char*)smem + L::LVL_BYTES);
	for (int l = tid; l < NLVL; l += 256) sLvl[l] = a.levels[l];
	__syncthreads();

	const _Float16* sW0 = smem + L::oW0;
	const _Float16* sW0T = smem + L::oW0T;
	const _Float16* sWh = smem + L::oWh;
	const _Float16* sWhT = smem + L::oWhT;
	const _Float16* sWo = smem + L::oWo;
	const _Float16* sWoT = smem + L::oWoT;
	_Float16* bufA = smem + L::oStage + wave * 2 * L::STAGE;
	_Float16* bufD = bufA + L::STAGE;

	f4 accWo[NT];
	f4 accH[NHM > 0 ? NHM : 1][NT][NT];
	f4 accW0[NT][NTI];
	const f4 fz = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
	for (int t = 0; t < NT; ++t) {
		accWo[t] = fz;
#pragma unroll
		for (int u = 0; u < NTI; ++u) accW0[t][u] = fz;
#pragma unroll
		for (int j = 0; j < (NHM > 0 ? NHM : 1); ++j)
#pragma unroll
			for (int u = 0; u < NT; ++u) accH[j][t][u] = fz;
	}
	float loss_acc = 0.0f;

	const bool hash_grid = a.hash_grid != 0;
	const Interp interp = (Interp)a.interp;
	const uint32_t n_chunks = a.B / 32;

	for (uint32_t chunk = blockIdx.x * 4 + wave; chunk < n_chunks; chunk += gridDim.x * 4) {
		const uint32_t base = chunk * 32;

		// ---------------- grid encoding -> B fragments (tiles of 4 features) ----------------
		h4 xt[2][NTI];
#pragma unroll
		for (int tau = 0; tau < 2; ++tau) {
			const uint32_t i = base + 16 * tau + c;
			float x[D];
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) x[d] = a.pos[(size_t)i * D + d];
#pragma unroll
			for (int s = 0; s < KI; ++s) {
#pragma unroll
				for (int pp = 0; pp < 4; ++pp) {
					const int level = 16 * s + 8 * (pp >> 1) + 2 * q + (pp & 1);
					const LevelInfo li = sLvl[level];
					const h2 e = encode_level_f2<D, H>(a.table, li, hash_grid, interp, x);
					xt[tau][2 * s + (pp >> 1)][2 * (pp & 1) + 0] = e[0];
					xt[tau][2 * s + (pp >> 1)][2 * (pp & 1) + 1] = e[1];
				}
			}
		}

		// ---------------- forward ----------------
		h4 act[NH][2][NT];
		{
			f4 acc[2][NT];
#pragma unroll
			for (int t = 0; t < NT; ++t) {
				acc[0][t] = fz; acc[1][t] = fz;
#pragma unroll
				for (int s = 0; s < KI; ++s) {
					const h8 af = lds_afrag(sW0, L::RSI, 16 * t + c, 32 * s + 4 * q);
					acc[0][t] = mfma16(af, cat8(xt[0][2 * s], xt[0][2 * s + 1]), acc[0][t]);
					acc[1][t] = mfma16(af, cat8(xt[1][2 * s], xt[1][2 * s + 1]), acc[1][t]);
				}
			}
#pragma unroll
			for (int t = 0; t < NT; ++t) { act[0][0][t] = act_fwd<ACT>(acc[0][t]); act[0][1][t] = act_fwd<ACT>(acc[1][t]); }
		}
#pragma unroll
		for (int j = 1; j < NH; ++j) {
			const _Float16* Wm = sWh + (j - 1) * W * L::RSW;
			f4 acc[2][NT];
#pragma unroll
			for (int t = 0; t < NT; ++t) {
				acc[0][t] = fz; acc[1][t] = fz;
#pragma unroll
				for (int s = 0; s < KW; ++s) {
					const h8 af = lds_afrag(Wm, L::RSW, 16 * t + c, 32 * s + 4 * q);
					acc[0][t] = mfma16(af, cat8(act[j - 1][0][2 * s], act[j - 1][0][2 * s + 1]), acc[0][t]);
					acc[1][t] = mfma16(af, cat8(act[j - 1][1][2 * s], act[j - 1][1][2 * s + 1]), acc[1][t]);
				}
			}
#pragma unroll
			for (int t = 0; t < NT; ++t) { act[j][0][t] = act_fwd<ACT>(acc[0][t]); act[j][1][t] = act_fwd<ACT>(acc[1][t]); }
		}
		h4 G[2];
		{
			f4 yacc[2] = {fz, fz};
#pragma unroll
			for (int s = 0; s < KW; ++s) {
				const h8 af = lds_afrag(sWo, L::RSW, c, 32 * s + 4 * q);
				yacc[0] = mfma16(af, cat8(act[NH - 1][0][2 * s], act[NH - 1][0][2 * s + 1]), yacc[0]);
				yacc[1] = mfma16(af, cat8(act[NH - 1][1][2 * s], act[NH - 1][1][2 * s + 1]), yacc[1]);
			}
			// ---------------- RelativeL2 loss (relative_l2.h:40-76) ----------------
#pragma unroll
			for (int tau = 0; tau < 2; ++tau) {
				const uint32_t i = base + 16 * tau + c;
				if constexpr (EXT_DOUT) {
					G[tau] = *(const h4*)(a.dout + (size_t)i * 16 + 4 * q);
					continue;
				}
				const h4 y = __builtin_convertvector(yacc[tau], h4);
				if (a.out) *(h4*)(a.out + (size_t)i * 16 + 4 * q) = y;
				h4 g = zero4();
#pragma unroll
				for (int r = 0; r < 4; ++r) {
					const uint32_t o = 4 * q + r;
					if (o < a.dims) {
						const float p = (float)y[r];
						const float pse = __builtin_fmaf(p, p, 0.01f);
						const float d = p - a.target[(size_t)i * a.dims + o];
						loss_acc += d * d / pse / a.n_total;
						const float gr = 2.0f * d / pse;
						g[r] = (_Float16)(a.loss_scale * gr / a.n_total);
					}
				}
				G[tau] = g;
			}
		}

		// ---------------- backward + weight gradients ----------------
		// output layer: dWout += G * act[NH-1]^T
#pragma unroll
		for (int tau = 0; tau < 2; ++tau) {
			*(h4*)(bufD + (16 * tau + c) * L::RSS + 4 * q) = G[tau];
#pragma unroll
			for (int t = 0; t < NT; ++t) *(h4*)(bufA + (16 * tau + c) * L::RSS + 16 * t + 4 * q) = act[NH - 1][tau][t];
		}
		lds_fence();
		{
			const h8 ga = lds_trfrag(bufD, L::RSS, q, c, 0);
#pragma unroll
			for (int nt = 0; nt < NT; ++nt) accWo[nt] = mfma16(ga, lds_trfrag(bufA, L::RSS, q, c, nt), accWo[nt]);
		}
		h4 dl[2][NT];
#pragma unroll
		for (int t = 0; t < NT; ++t) {
			const h8 af = cat8(*(const h4*)(sWoT + (16 * t + c) * L::RSO + 4 * q), zero4());
			dl[0][t] = act_bwd<ACT>(act[NH - 1][0][t], mfma16(af, cat8(G[0], zero4()), fz));
			dl[1][t] = act_bwd<ACT>(act[NH - 1][1][t], mfma16(af, cat8(G[1], zero4()), fz));
		}
#pragma unroll
		for (int j = NH - 1; j >= 1; --j) {
			lds_fence();
#pragma unroll
			for (int tau = 0; tau < 2; ++tau) {
#pragma unroll
				for (int t = 0; t < NT; ++t) {
					*(h4*)(bufD + (16 * tau + c) * L::RSS + 16 * t + 4 * q) = dl[tau][t];
					*(h4*)(bufA + (16 * tau + c) * L::RSS + 16 * t + 4 * q) = act[j - 1][tau][t];
				}
			}
			lds_fence();
			{
				h8 bf[NT];
#pragma unroll
				for (int nt = 0; nt < NT; ++nt) bf[nt] = lds_trfrag(bufA, L::RSS, q, c, nt);
#pragma unroll
				for (int mt = 0; mt < NT; ++mt) {
					const h8 ad = lds_trfrag(bufD, L::RSS, q, c, mt);
#pragma unroll
					for (int nt = 0; nt < NT; ++nt) accH[j - 1][mt][nt] = mfma16(ad, bf[nt], accH[j - 1][mt][nt]);
				}
			}
			const _Float16* WT = sWhT + (j - 1) * W * L::RSW;
			h4 ndl[2][NT];
#pragma unroll
			for (int t = 0; t < NT; ++t) {
				f4 acc0 = fz, acc1 = fz;
#pragma unroll
				for (int s = 0; s < KW; ++s) {
					const h8 af = lds_afrag(WT, L::RSW, 16 * t + c, 32 * s + 4 * q);
					acc0 = mfma16(af, cat8(dl[0][2 * s], dl[0][2 * s + 1]), acc0);
					acc1 = mfma16(af, cat8(dl[1][2 * s], dl[1][2 * s + 1]), acc1);
				}
				ndl[0][t] = act_bwd<ACT>(act[j - 1][0][t], acc0);
				ndl[1][t] = act_bwd<ACT>(act[j - 1][1][t], acc1);
			}
#pragma unroll
			for (int t = 0; t < NT; ++t) { dl[0][t] = ndl[0][t]; dl[1][t] = ndl[1][t]; }
		}
		// first layer: dW0 += dl * x^T ; dL/dx = W0^T dl
		lds_fence();
#pragma unroll
		for (int tau = 0; tau < 2; ++tau) {
#pragma unroll
			for (int t = 0; t < NT; ++t) *(h4*)(bufD + (16 * tau + c) * L::RSS + 16 * t + 4 * q) = dl[tau][t];
#pragma unroll
			for (int u = 0; u < NTI; ++u) *(h4*)(bufA + (16 * tau + c) * L::RSS + 16 * u + 4 * q) = xt[tau][u];
		}
		lds_fence();
		{
			h8 bf[NTI];
#pragma unroll
			for (int u = 0; u < NTI; ++u) bf[u] = lds_trfrag(bufA, L::RSS, q, c, u);
#pragma unroll
			for (int mt = 0; mt < NT; ++mt) {
				const h8 ad = lds_trfrag(bufD, L::RSS, q, c, mt);
#pragma unroll
				for (int u = 0; u < NTI; ++u) accW0[mt][u] = mfma16(ad, bf[u], accW0[mt][u]);
			}
		}
#pragma unroll
		for (int u = 0; u < NTI; ++u) {
			f4 acc0 = fz, acc1 = fz;
#pragma unroll
			for (int s = 0; s < KW; ++s) {
				const h8 af = lds_afrag(sW0T, L::RSW, 16 * u + c, 32 * s + 4 * q);
				acc0 = mfma16(af, cat8(dl[0][2 * s], dl[0][2 * s + 1]), acc0);
				acc1 = mfma16(af, cat8(dl[1][2 * s], dl[1][2 * s + 1]), acc1);
			}
			const h4 d0 = __builtin_convertvector(acc0, h4);
			const h4 d1 = __builtin_convertvector(acc1, h4);
			const uint32_t lv = 8 * u + 2 * q;  // features 16u + 4q + r -> levels lv (r=0,1), lv+1 (r=2,3)
			const uint32_t i0 = base + c, i1 = base + 16 + c;
			a.dLdenc[(size_t)lv * a.B + i0] = __builtin_bit_cast(uint32_t, h2{d0[0], d0[1]});
			a.dLdenc[(size_t)(lv + 1) * a.B + i0] = __builtin_bit_cast(uint32_t, h2{d0[2], d0[3]});
			a.dLdenc[(size_t)lv * a.B + i1] = __builtin_bit_cast(uint32_t, h2{d1[0], d1[1]});
			a.dLdenc[(size_t)(lv + 1) * a.B + i1] = __builtin_bit_cast(uint32_t, h2{d1[2], d1[3]});
		}
	}

	// ---------------- workgroup reduction of dW and loss -> partial slabs ----------------
	// Waves add their register accumulators into one LDS slab in fixed wave order (plain LDS
	// loads/stores: gfx950 LDS float atomics are ~24x slower than integer ones, and a fixed order
	// keeps the partial bit-reproducible).
	__syncthreads();
	float* red = (float*)smem;
	constexpr int oH = W * IN, oO = W * IN + NHM * W * W;
#pragma unroll
	for (int off = 32; off > 0; off >>= 1) loss_acc += __shfl_xor(loss_acc, off);
	for (int w = 0; w < 4; ++w) {
		if (wave == w) {
			const bool first = (w == 0);
#pragma unroll
			for (int mt = 0; mt < NT; ++mt) {
#pragma unroll
				for (int r = 0; r < 4; ++r) {
					const int n = 16 * mt + 4 * q + r;
#pragma unroll
					for (int u = 0; u < NTI; ++u) {
						float* p = &red[n * IN + 16 * u + c];
						*p = first ? accW0[mt][u][r] : *p + accW0[mt][u][r];
					}
#pragma unroll
					for (int j = 0; j < NHM; ++j)
#pragma unroll
						for (int nt = 0; nt < NT; ++nt) {
							float* p = &red[oH + j * W * W + n * W + 16 * nt + c];
							*p = first ? accH[j][mt][nt][r] : *p + accH[j][mt][nt][r];
						}
				}
			}
#pragma unroll
			for (int nt = 0; nt < NT; ++nt)
#pragma unroll
				for (int r = 0; r < 4; ++r) {
					float* p = &red[oO + (4 * q + r) * W + 16 * nt + c];
					*p = first ? accWo[nt][r] : *p + accWo[nt][r];
				}
			if (lane == 0) red[L::N_MLP + w] = loss_acc;
		}
		__syncthreads();
	}
	float* dst = a.wgrad_partial + (size_t)blockIdx.x * L::N_MLP;
	for (int p = tid; p < L::N_MLP; p += 256) dst[p] = red[p];
	if (tid == 0) a.loss_partial[blockIdx.x] = red[L::N_MLP] + red[L::N_MLP + 1] + red[L::N_MLP + 2] + red[L::N_MLP + 3];
}


// Forward-only pass (inference / forward context): input fp16 from memory, SoA ([IN][B], the grid
// encoding's layout) or AoS ([B][IN]); output fp16 [B][16] (the reference's CM [16 x B]).
// Reference: kernel_mlp_fused<..., INFERENCE=true> (fully_fused_mlp.cu:499-557).
template <int W, int IN, int NH, Act ACT, bool SOA>
__global__ __launch_bounds__(256, 2) void k_mlp_infer(uint32_t B, const _Float16* __restrict__ wimage,
                                                      const _Float16* __restrict__ in, _Float16* __restrict__ out) {
	using L = FusedLayout<W, IN, NH>;
	constexpr int NT = L::NT, KW = L::KW, NTI = L::NTI, KI = L::KI;
	extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
	const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	const int c = lane & 15, q = lane >> 4;
	copy_image_to_lds(smem, wimage, L::oStage, tid, 256);
	__syncthreads();
	const _Float16* sW0 = smem + L::oW0;
	const _Float16* sWh = smem + L::oWh;
	const _Float16* sWo = smem + L::oWo;
	const f4 fz = {0.0f, 0.0f, 0.0f, 0.0f};
	const uint32_t n_chunks = B / 16;
	for (uint32_t chunk = blockIdx.x * 4 + wave; chunk < n_chunks; chunk += gridDim.x * 4) {
		const uint32_t i = chunk * 16 + c;
		h4 xt[NTI];
#pragma unroll
		for (int u = 0; u < NTI; ++u) {
#pragma unroll
			for (int r = 0; r < 4; ++r) {
				const uint32_t f = 16 * u + 4 * q + r;
				xt[u][r] = SOA ? in[(size_t)f * B + i] : in[(size_t)i * IN + f];
			}
		}
		h4 act[NT];
		{
			f4 acc[NT];
#pragma unroll
			for (int t = 0; t < NT; ++t) {
				acc[t] = fz;
#pragma unroll
				for (int s = 0; s < KI; ++s) acc[t] = mfma16(lds_afrag(sW0, L::RSI, 16 * t + c, 32 * s + 4 * q), cat8(xt[2 * s], xt[2 * s + 1]), acc[t]);
			}
#pragma unroll
			for (int t = 0; t < NT; ++t) act[t] = act_fwd<ACT>(acc[t]);
		}
#pragma unroll
		for (int j = 1; j < NH; ++j) {
			const _Float16* Wm = sWh + (j - 1) * W * L::RSW;
			f4 acc[NT];
#pragma unroll
			for (int t = 0; t < NT; ++t) {
				acc[t] = fz;
#pragma unroll
				for (int s = 0; s < KW; ++s) acc[t] = mfma16(lds_afrag(Wm, L::RSW, 16 * t + c, 32 * s + 4 * q), cat8(act[2 * s], act[2 * s + 1]), acc[t]);
			}
#pragma unroll
			for (int t = 0; t < NT; ++t) act[t] = act_fwd<ACT>(acc[t]);
		}
		f4 y = fz;
#pragma unroll
		for (int s = 0; s < KW; ++s) y = mfma16(lds_afrag(sWo, L::RSW, c, 32 * s + 4 * q), cat8(act[2 * s], act[2 * s + 1]), y);
		*(h4*)(out + (size_t)i * 16 + 4 * q) = __builtin_convertvector(y, h4);
	}
}

}  // namespace tcnn_amd
