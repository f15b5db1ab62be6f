// mlp_tile.hip -- fully fused MLP training for the shapes the register-resident kernel
// (mlp_fused.h: W <= 64, grid input, two hidden layers) cannot hold: W in {64, 128}, any input
// encoding (hash grid, OneBlob, Identity) read as fp16 [B][IN], IN <= 128.
//
// Reference: kernel_mlp_fused / kernel_mlp_fused_backward (fully_fused_mlp.cu:47-259, 499-557) and
// the CUTLASS weight-gradient GEMMs (fully_fused_mlp.cu:735-836). The reference writes every hidden
// activation and every backprop temporary to HBM ([W x B] fp16 per layer, twice) and reads them back
// for the split-K weight gradients; for W128/H4 at B = 2^20 that is ~5 KB per sample. Here one
// workgroup owns the whole network for 32-sample tiles:
//   * all weights are staged once into LDS (W128/H4/IN32: 119 KB, padded rows, fp16);
//   * a tile's input and its NH post-activations stay in LDS ([32][W+8] fp16 per layer, 35 KB) for
//     the backward pass, the loss is fused after the output layer, and each backprop delta
//     overwrites the activation slot it no longer needs;
//   * weight gradients accumulate in registers across all tiles the workgroup processes: wave w owns
//     output-row tiles w*W/64 .. of every matrix (the MFMA contracts over the 32 samples of a tile,
//     operands read from LDS with the gfx950 ds_read_b64_tr_b16 transpose read), so no cross-wave
//     reduction exists; one fp32 partial slab per workgroup leaves at the end;
//   * dL/d(encoding) = W0^T delta_1 leaves in the layout the grid backward reads (level-major
//     feature pairs) or AoS for the OneBlob / Identity input gradient.
// One workgroup of 4 waves per CU (the LDS is full), persistent over the tiles; fp32 MFMA
// accumulation (f32_16x16x32_f16), fp16 storage at the reference's points.
#include "kernels.h"
#include "mlp_fused.h"

namespace tcnn_amd {

// LDS halves of a tile workgroup with the first NS hidden matrices streamed from L2 instead of staged
constexpr int tile_halves(int W, int IN, int NH, int NS) {
	const int KP0 = (IN + 31) / 32 * 32, RS0 = KP0 + 8, RSW = W + 8, RSG = 24;
	return W * RS0 + (NH - 1 - NS) * W * RSW + 16 * RSW + 32 * RS0 + NH * 32 * RSW + 32 * RSG;
}
// W128 runs 8 waves (2 per SIMD, one 16-row tile of every matrix each) up to 4 hidden layers; with 5
// its weight-gradient accumulators (>= 164 registers) spill at 256 registers per wave, so it runs 4
// waves (1 per SIMD, 512 registers incl. AGPRs, two row tiles each: half the activation LDS reads)
constexpr int tile_waves(int W, int NH) { return W == 128 && NH < 5 ? 8 : 4; }
constexpr int tile_lds_limit() { return 160 * 1024; }
// fewest streamed hidden matrices that let the rest of the network + the tile's activations fit
constexpr int tile_n_streamed(int W, int IN, int NH) {
	int ns = 0;
	while (ns < NH - 1 && tile_halves(W, IN, NH, ns) * 2 + tile_waves(W, NH) * 4 > tile_lds_limit()) ++ns;
	return ns;
}

template <int W, int IN, int NH>
struct TileLayout {
	static_assert(W == 64 || W == 128, "tile engine: W in {64, 128}");
	static_assert(IN % 16 == 0 && IN <= 128, "tile engine: IN a multiple of 16, <= 128");
	static constexpr int KP0 = (IN + 31) / 32 * 32;  // K of the first layer, padded to the MFMA depth
	static constexpr int RS0 = KP0 + 8, RSW = W + 8, RSG = 24;
	static constexpr int WAVES = tile_waves(W, NH), NTHR = WAVES * 64;
	static constexpr int MT = W / 16, MTW = MT / WAVES;  // output-row tiles per matrix / per wave
	static constexpr int KT0 = IN / 16;              // feature tiles of the input
	// hidden matrices 1..NS are not staged: their forward A fragments come from the fp16 parameters
	// (L2-resident, every workgroup reads the same 32 KB), their backward ones from a transposed copy
	static constexpr int NS = tile_n_streamed(W, IN, NH);
	static constexpr int oW0 = 0, oWh = oW0 + W * RS0, oWo = oWh + (NH - 1 - NS) * W * RSW;
	static constexpr int oX = oWo + 16 * RSW;                 // slot 0: the tile's input [32][RS0]
	static constexpr int oA = oX + 32 * RS0;                  // slots 1..NH: [32][RSW]
	static constexpr int oG = oA + NH * 32 * RSW;             // dL/dy of the tile [32][RSG]
	static constexpr int HALVES = oG + 32 * RSG;
	static constexpr int BYTES = HALVES * 2 + WAVES * 4;       // + per-wave loss
	static constexpr int N_MLP = W * IN + (NH - 1) * W * W + 16 * W;
	static_assert(HALVES == tile_halves(W, IN, NH, NS), "layout");
	static_assert(oWh % 8 == 0 && oWo % 8 == 0 && oX % 8 == 0 && oA % 8 == 0 && oG % 8 == 0, "16-byte alignment");
};

struct TileTrainArgs {
	uint32_t B, dims, loss_l2;
	float loss_scale, n_total;
	const _Float16* params;  // [W0 | hidden | Wout] fp16
	const _Float16* wT;      // streamed hidden matrices 1..NS transposed, [NS][W (in)][W (out)] fp16
	const _Float16* enc;     // encoded input fp16 [B][IN]
	const float* target;     // [B][dims] (loss)
	const _Float16* dout;    // external dL/d(output) fp16 [B][16] (EXT_DOUT, loss-scaled by the caller)
	_Float16* out;           // optional network output fp16 [B][16]
	void* dldenc;            // optional dL/d(encoding): pairs [IN/2][B] (uint32) or AoS fp16 [B][IN]
	int dldenc_pairs;
	float* wgrad_partial;    // [gridDim.x][N_MLP]
	float* loss_partial;     // [gridDim.x]
};

__device__ __forceinline__ h8 zero8() { return h8{0, 0, 0, 0, 0, 0, 0, 0}; }

template <Act ACT>
__device__ __forceinline__ h4 tile_act(f4 v) {
	return act_fwd<ACT>(v);
}

template <int W, int IN, int NH, Act ACT, bool EXT_DOUT>
__global__ __launch_bounds__(tile_waves(W, NH) * 64, 1) void k_mlp_tile_train(const TileTrainArgs a) {
	using L = TileLayout<W, IN, NH>;
	constexpr int MTW = L::MTW, KT0 = L::KT0, RS0 = L::RS0, RSW = L::RSW, RSG = L::RSG;
	constexpr int WAVES = L::WAVES, NTHR = L::NTHR;
	constexpr int NTW = L::MT / WAVES;  // Wout column tiles per wave (= MTW)
	extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
	const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	const int c = lane & 15, q = lane >> 4;
	const f4 fz = {0.0f, 0.0f, 0.0f, 0.0f};
	float* wloss = (float*)(smem + L::HALVES);

	// ---- weights -> LDS (rows padded; first-layer columns [IN, KP0) zero) ----
	{
		const _Float16* p = a.params;
		for (int idx = tid; idx < W * (L::KP0 / 8); idx += NTHR) {
			const int r = idx / (L::KP0 / 8), c8 = idx % (L::KP0 / 8);
			*(h8*)(smem + L::oW0 + r * RS0 + 8 * c8) = 8 * c8 < IN ? *(const h8*)(p + (size_t)r * IN + 8 * c8) : zero8();
		}
		p += W * IN;
		for (int idx = tid; idx < (NH - 1 - L::NS) * W * (W / 8); idx += NTHR) {
			const int r = idx / (W / 8), c8 = idx % (W / 8);  // r over the staged hidden rows
			*(h8*)(smem + L::oWh + r * RSW + 8 * c8) = *(const h8*)(p + (size_t)(L::NS * W + r) * W + 8 * c8);
		}
		p += (NH - 1) * W * W;
		for (int idx = tid; idx < 16 * (W / 8); idx += NTHR) {
			const int r = idx / (W / 8), c8 = idx % (W / 8);
			*(h8*)(smem + L::oWo + r * RSW + 8 * c8) = *(const h8*)(p + (size_t)r * W + 8 * c8);
		}
		// zero the padded input columns of slot 0 once (the input loads never write them)
		if (L::KP0 > IN)
			for (int idx = tid; idx < 32 * (L::KP0 - IN); idx += NTHR)
				smem[L::oX + (idx / (L::KP0 - IN)) * RS0 + IN + idx % (L::KP0 - IN)] = (_Float16)0.0f;
	}
	// staged matrices (m == 0 or m > NS); streamed ones (1 <= m <= NS) are read from global memory
	auto Wm = [&](int m) -> const _Float16* { return m == 0 ? smem + L::oW0 : smem + L::oWh + (m - 1 - L::NS) * W * RSW; };
	auto streamed = [](int m) { return m >= 1 && m <= L::NS; };
	auto slot = [&](int m) -> _Float16* { return m == 0 ? smem + L::oX : smem + L::oA + (m - 1) * 32 * RSW; };
	_Float16* sG = smem + L::oG;

	// ---- register accumulators of this wave's weight-gradient rows ----
	f4 dW0[MTW][KT0];
	f4 dWh[NH > 1 ? NH - 1 : 1][MTW][L::MT];
	f4 dWo[NTW];
#pragma unroll
	for (int i = 0; i < MTW; ++i) {
#pragma unroll
		for (int k = 0; k < KT0; ++k) dW0[i][k] = fz;
#pragma unroll
		for (int j = 0; j < (NH > 1 ? NH - 1 : 1); ++j)
#pragma unroll
			for (int k = 0; k < L::MT; ++k) dWh[j][i][k] = fz;
	}
#pragma unroll
	for (int i = 0; i < NTW; ++i) dWo[i] = fz;
	float loss = 0.0f;

	// input rows of a tile: IN/8 16-byte vectors per sample
	constexpr int XV = 32 * IN / 8, XPT = (XV + NTHR - 1) / NTHR;
	const uint32_t n_tiles = a.B / 32;
	uint32_t tile = blockIdx.x;
	h8 xr[XPT];
	auto load_x = [&](uint32_t t) {
#pragma unroll
		for (int j = 0; j < XPT; ++j) {
			const int idx = tid + NTHR * j;
			if (idx < XV) xr[j] = *(const h8*)(a.enc + ((size_t)t * 32 + idx / (IN / 8)) * IN + 8 * (idx % (IN / 8)));
		}
	};
	if (tile < n_tiles) load_x(tile);
	__syncthreads();

	for (; tile < n_tiles; tile += gridDim.x) {
		const uint32_t base = tile * 32;
		// ---- input tile -> slot 0; prefetch the next tile's rows ----
#pragma unroll
		for (int j = 0; j < XPT; ++j) {
			const int idx = tid + NTHR * j;
			if (idx < XV) *(h8*)(slot(0) + (idx / (IN / 8)) * RS0 + 8 * (idx % (IN / 8))) = xr[j];
		}
		if (tile + gridDim.x < n_tiles) load_x(tile + gridDim.x);
		// targets / external dL/dy of this wave's output lanes (waves 0, 1: sample tile tau = wave)
		float tg[4] = {0.0f, 0.0f, 0.0f, 0.0f};
		h4 gext = zero4();
		if (wave < 2) {
			const uint32_t i = base + 16 * wave + c;
			if constexpr (EXT_DOUT) {
				gext = *(const h4*)(a.dout + (size_t)i * 16 + 4 * q);
			} else {
#pragma unroll
				for (int r = 0; r < 4; ++r)
					if (4 * q + r < (int)a.dims) tg[r] = a.target[(size_t)i * a.dims + 4 * q + r];
			}
		}
		__syncthreads();

		// ---- forward: a_{m+1} = act(M_m a_m), this wave's output-row tiles ----
#pragma unroll
		for (int m = 0; m < NH; ++m) {
			const int KS = (m == 0 ? L::KP0 : W) / 32;
			const int rsi = m == 0 ? RS0 : RSW;
			const _Float16* Wt = streamed(m) ? nullptr : Wm(m);
			const _Float16* in = slot(m);
			f4 acc[MTW][2];
#pragma unroll
			for (int i = 0; i < MTW; ++i) acc[i][0] = acc[i][1] = fz;
			h8 ag[MTW][W / 32];  // a streamed layer's A fragments, all loads issued before the first MFMA
			if (streamed(m)) {
				const _Float16* Wg = a.params + (size_t)W * IN + (size_t)(m - 1) * W * W;
#pragma unroll
				for (int i = 0; i < MTW; ++i)
#pragma unroll
					for (int s = 0; s < W / 32; ++s) ag[i][s] = *(const h8*)(Wg + (size_t)(16 * (wave * MTW + i) + c) * W + 32 * s + 8 * q);
			}
#pragma unroll
			for (int s = 0; s < KS; ++s) {
				const h8 b0 = *(const h8*)(in + c * rsi + 32 * s + 8 * q);
				const h8 b1 = *(const h8*)(in + (16 + c) * rsi + 32 * s + 8 * q);
#pragma unroll
				for (int i = 0; i < MTW; ++i) {
					const h8 af = streamed(m) ? ag[i][s] : *(const h8*)(Wt + (16 * (wave * MTW + i) + c) * rsi + 32 * s + 8 * q);
					acc[i][0] = mfma16(af, b0, acc[i][0]);
					acc[i][1] = mfma16(af, b1, acc[i][1]);
				}
			}
			_Float16* outs = slot(m + 1);
#pragma unroll
			for (int i = 0; i < MTW; ++i)
#pragma unroll
				for (int tau = 0; tau < 2; ++tau)
					*(h4*)(outs + (16 * tau + c) * RSW + 16 * (wave * MTW + i) + 4 * q) = tile_act<ACT>(acc[i][tau]);
			__syncthreads();
		}

		// ---- output layer + loss (waves 0, 1: sample tile tau = wave) ----
		if (wave < 2) {
			const int tau = wave;
			const _Float16* aN = slot(NH);
			f4 y = fz;
#pragma unroll
			for (int s = 0; s < W / 32; ++s)
				y = mfma16(*(const h8*)(smem + L::oWo + c * RSW + 32 * s + 8 * q), *(const h8*)(aN + (16 * tau + c) * RSW + 32 * s + 8 * q), y);
			const uint32_t i = base + 16 * tau + c;
			const h4 yh = __builtin_convertvector(y, h4);
			if (a.out) *(h4*)(a.out + (size_t)i * 16 + 4 * q) = yh;
			h4 g = zero4();
			if constexpr (EXT_DOUT) {
				g = gext;
			} else {
#pragma unroll
				for (int r = 0; r < 4; ++r) {
					const uint32_t o = 4 * q + r;
					if (o < a.dims) {
						const float p = (float)yh[r];
						const float pse = a.loss_l2 ? 1.0f : __builtin_fmaf(p, p, 0.01f);  // relative_l2.h:67-75 / l2.h:66-74
						const float d = p - tg[r];
						loss += d * d / pse / a.n_total;
						g[r] = f16_rn(a.loss_scale * (2.0f * d / pse) / a.n_total);
					}
				}
			}
			*(h4*)(sG + (16 * tau + c) * RSG + 4 * q) = g;
		}
		__syncthreads();

		// ---- dWout += G^T a_NH ; delta_NH = act'(a_NH) * (Wout^T G) ----
		h4 dl[MTW][2];
		{
			const _Float16* aN = slot(NH);
			const h8 ga = lds_trfrag(sG, RSG, q, c, 0);  // A[out c][sample 8q+e]
#pragma unroll
			for (int i = 0; i < NTW; ++i) dWo[i] = mfma16(ga, lds_trfrag(aN, RSW, q, c, wave * NTW + i), dWo[i]);
			h8 gb[2];
#pragma unroll
			for (int tau = 0; tau < 2; ++tau) gb[tau] = q < 2 ? *(const h8*)(sG + (16 * tau + c) * RSG + 8 * q) : zero8();
#pragma unroll
			for (int i = 0; i < MTW; ++i) {
				const int mt = wave * MTW + i;
				// A[neuron][out 8q+e]: K = 16 outputs, the upper half of the MFMA depth is zero through gb.
				// Every lane takes part in the transpose read (lanes q >= 2 re-read rows 0..15): the
				// ds_read_b64_tr_b16 exchange under a partial EXEC mask returned garbage (NaN deltas).
				const h8 af = lds_trfrag(smem + L::oWo, RSW, q & 1, c, mt);
#pragma unroll
				for (int tau = 0; tau < 2; ++tau) {
					const f4 v = mfma16(af, gb[tau], fz);
					dl[i][tau] = act_bwd<ACT>(*(const h4*)(aN + (16 * tau + c) * RSW + 16 * mt + 4 * q), v);
				}
			}
		}
		__syncthreads();
		{
			_Float16* aN = slot(NH);
#pragma unroll
			for (int i = 0; i < MTW; ++i)
#pragma unroll
				for (int tau = 0; tau < 2; ++tau) *(h4*)(aN + (16 * tau + c) * RSW + 16 * (wave * MTW + i) + 4 * q) = dl[i][tau];
		}
		__syncthreads();

		// ---- hidden layers and the first layer, last to first ----
#pragma unroll
		for (int m = NH - 1; m >= 0; --m) {
			const _Float16* dsl = slot(m + 1);  // delta_{m+1} [sample][neuron]
			const _Float16* am = slot(m);       // a_m [sample][feature]
			const int rsm = m == 0 ? RS0 : RSW;
			// a streamed matrix's transposed A fragments (A[feature][neuron] = M^T rows of this wave's
			// tiles), loaded ahead so the latency hides behind the weight-gradient MFMAs
			h8 agT[MTW][W / 32];
			if (streamed(m)) {
				const _Float16* WgT = a.wT + (size_t)(m - 1) * W * W;
#pragma unroll
				for (int i = 0; i < MTW; ++i)
#pragma unroll
					for (int s = 0; s < W / 32; ++s) agT[i][s] = *(const h8*)(WgT + (size_t)(16 * (wave * MTW + i) + c) * W + 32 * s + 8 * q);
			}
			// dW_m += delta_{m+1} a_m^T (contraction over the tile's 32 samples)
#pragma unroll
			for (int i = 0; i < MTW; ++i) {
				const h8 ad = lds_trfrag(dsl, RSW, q, c, wave * MTW + i);  // A[neuron][sample]
				if (m == 0) {
#pragma unroll
					for (int k = 0; k < KT0; ++k) dW0[i][k] = mfma16(ad, lds_trfrag(am, rsm, q, c, k), dW0[i][k]);
				} else {
#pragma unroll
					for (int k = 0; k < L::MT; ++k) dWh[m > 0 ? m - 1 : 0][i][k] = mfma16(ad, lds_trfrag(am, rsm, q, c, k), dWh[m > 0 ? m - 1 : 0][i][k]);
				}
			}
			// delta_m = act'(a_m) * (M_m^T delta_{m+1})  (m == 0: dL/d(encoding), no transfer)
			const _Float16* Mt = streamed(m) ? nullptr : Wm(m);
			if (m > 0) {
#pragma unroll
				for (int i = 0; i < MTW; ++i) {
					const int t = wave * MTW + i;
					f4 v0 = fz, v1 = fz;
#pragma unroll
					for (int s = 0; s < W / 32; ++s) {
						const h8 af = streamed(m) ? agT[i][s] : lds_trfrag(Mt + 32 * s * rsm, rsm, q, c, t);  // A[feature][neuron 32s+8q+e]
						v0 = mfma16(af, *(const h8*)(dsl + c * RSW + 32 * s + 8 * q), v0);
						v1 = mfma16(af, *(const h8*)(dsl + (16 + c) * RSW + 32 * s + 8 * q), v1);
					}
					dl[i][0] = act_bwd<ACT>(*(const h4*)(am + c * rsm + 16 * t + 4 * q), v0);
					dl[i][1] = act_bwd<ACT>(*(const h4*)(am + (16 + c) * rsm + 16 * t + 4 * q), v1);
				}
				__syncthreads();
				_Float16* dst = slot(m);  // a_m is dead: delta_m takes its slot
#pragma unroll
				for (int i = 0; i < MTW; ++i)
#pragma unroll
					for (int tau = 0; tau < 2; ++tau) *(h4*)(dst + (16 * tau + c) * RSW + 16 * (wave * MTW + i) + 4 * q) = dl[i][tau];
				__syncthreads();
			} else if (a.dldenc) {
				for (int t = wave; t < KT0; t += WAVES) {
					f4 v[2] = {fz, fz};
#pragma unroll
					for (int s = 0; s < W / 32; ++s) {
						const h8 af = lds_trfrag(Mt + 32 * s * RS0, RS0, q, c, t);
#pragma unroll
						for (int tau = 0; tau < 2; ++tau) v[tau] = mfma16(af, *(const h8*)(dsl + (16 * tau + c) * RSW + 32 * s + 8 * q), v[tau]);
					}
#pragma unroll
					for (int tau = 0; tau < 2; ++tau) {
						const h4 d = __builtin_convertvector(v[tau], h4);
						const uint32_t i = base + 16 * tau + c;
						if (a.dldenc_pairs) {  // features 16t + 4q + r -> levels 8t + 2q (r = 0, 1), + 1 (r = 2, 3)
							uint32_t* d2 = (uint32_t*)a.dldenc;
							const uint32_t lv = 8 * t + 2 * q;
							d2[(size_t)lv * a.B + i] = __builtin_bit_cast(uint32_t, h2{d[0], d[1]});
							d2[(size_t)(lv + 1) * a.B + i] = __builtin_bit_cast(uint32_t, h2{d[2], d[3]});
						} else {
							*(h4*)((_Float16*)a.dldenc + (size_t)i * IN + 16 * t + 4 * q) = d;
						}
					}
				}
				__syncthreads();
			} else {
				__syncthreads();
			}
		}
	}

	// ---- this workgroup's weight-gradient partial slab (each parameter owned by one lane) ----
	float* dst = a.wgrad_partial + (size_t)blockIdx.x * L::N_MLP;
#pragma unroll
	for (int i = 0; i < MTW; ++i) {
#pragma unroll
		for (int r = 0; r < 4; ++r) {
			const int row = 16 * (wave * MTW + i) + 4 * q + r;
#pragma unroll
			for (int k = 0; k < KT0; ++k) dst[row * IN + 16 * k + c] = dW0[i][k][r];
#pragma unroll
			for (int j = 0; j < NH - 1; ++j)
#pragma unroll
				for (int k = 0; k < L::MT; ++k) dst[W * IN + j * W * W + row * W + 16 * k + c] = dWh[j][i][k][r];
		}
	}
#pragma unroll
	for (int i = 0; i < NTW; ++i)
#pragma unroll
		for (int r = 0; r < 4; ++r) dst[W * IN + (NH - 1) * W * W + (4 * q + r) * W + 16 * (wave * NTW + i) + c] = dWo[i][r];
#pragma unroll
	for (int off = 32; off > 0; off >>= 1) loss += __shfl_xor(loss, off);
	if (lane == 0) wloss[wave] = loss;
	__syncthreads();
	if (tid == 0) {
		float l = 0.0f;
		for (int w = 0; w < WAVES; ++w) l += wloss[w];
		a.loss_partial[blockIdx.x] = l;
	}
}

// ------------------------------------------------------------------------------------------
// dispatch
// ------------------------------------------------------------------------------------------
#define TILE_SHAPES(X) \
	X(64, 16, 2) X(64, 16, 3) X(64, 16, 4) X(64, 16, 5) \
	X(64, 32, 1) X(64, 32, 2) X(64, 32, 3) X(64, 32, 4) X(64, 32, 5) \
	X(64, 64, 2) X(64, 64, 3) X(64, 64, 4) X(64, 64, 5) \
	X(64, 128, 2) X(64, 128, 3) X(64, 128, 4) X(64, 128, 5) \
	X(128, 16, 2) X(128, 16, 3) X(128, 16, 4) X(128, 16, 5) \
	X(128, 32, 1) X(128, 32, 2) X(128, 32, 3) X(128, 32, 4) X(128, 32, 5) \
	X(128, 64, 2) X(128, 64, 3) X(128, 64, 4) X(128, 64, 5) \
	X(128, 128, 2) X(128, 128, 3) X(128, 128, 4) X(128, 128, 5)

uint32_t tile_train_lds_bytes(uint32_t W, uint32_t IN, uint32_t NH) {
#define X(w, in, nh) \
	if (W == w && IN == in && NH == nh) return (uint32_t)TileLayout<w, in, nh>::BYTES;
	TILE_SHAPES(X)
#undef X
	return 0;
}

uint32_t tile_train_n_streamed(uint32_t W, uint32_t IN, uint32_t NH) {
#define X(w, in, nh) \
	if (W == w && IN == in && NH == nh) return (uint32_t)TileLayout<w, in, nh>::NS;
	TILE_SHAPES(X)
#undef X
	return 0;
}

uint32_t tile_train_wT_bytes(uint32_t W, uint32_t IN, uint32_t NH) { return tile_train_n_streamed(W, IN, NH) * W * W * 2; }

// transposed copy of the streamed hidden matrices 1..NS: wT[j][f][n] = M_{j+1}[n][f]
__global__ void k_tile_transpose_hidden(const _Float16* __restrict__ hidden, _Float16* __restrict__ wT, uint32_t W, uint32_t n) {
	const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
	if (idx >= n) return;
	const uint32_t j = idx / (W * W), r = idx % (W * W), f = r / W, o = r % W;
	wT[idx] = hidden[(size_t)j * W * W + (size_t)o * W + f];
}

bool tile_train_supported(uint32_t W, uint32_t IN, uint32_t NH, uint32_t outp, int act) {
	return outp == 16 && (act == ACT_NONE || act == ACT_RELU) && tile_train_lds_bytes(W, IN, NH) != 0 &&
	       tile_train_lds_bytes(W, IN, NH) <= 160 * 1024;
}

template <int W, int IN, int NH, Act ACT, bool EXT>
static void tile_launch(hipStream_t st, uint32_t blocks, const TileTrainArgs& a) {
	using L = TileLayout<W, IN, NH>;
	static bool attr = false;
	if (!attr) {
		TCNN_HIP_CHECK(hipFuncSetAttribute((const void*)k_mlp_tile_train<W, IN, NH, ACT, EXT>, hipFuncAttributeMaxDynamicSharedMemorySize,
		                                   (int)L::BYTES));
		attr = true;
	}
	hipLaunchKernelGGL((k_mlp_tile_train<W, IN, NH, ACT, EXT>), dim3(blocks), dim3(L::NTHR), L::BYTES, st, a);
}

// Workgroups per CU: 2 where the LDS holds two (the W64 shapes: a second workgroup hides the first's
// barrier and LDS latency at 1 wave per SIMD -- configs[1] 8,240 -> 10,468 steps/s, the sample's
// default 7,072 -> 9,380; 3 measured mixed, profiles/r02_tile_wg_per_cu.txt), capped by the LDS fit.
// TCNN_TILE_WG_PER_CU overrides (A/B switch).
uint32_t tile_train_blocks(uint32_t B, uint32_t W, uint32_t IN, uint32_t NH) {
	static const uint32_t want = [] {
		const char* e = std::getenv("TCNN_TILE_WG_PER_CU");
		return e ? std::max(1u, (uint32_t)std::atoi(e)) : 2u;
	}();
	const uint32_t bytes = tile_train_lds_bytes(W, IN, NH);
	const uint32_t fit = bytes ? std::max(1u, (160u * 1024u) / bytes) : 1u;
	return std::max(1u, std::min(256u * std::min(want, fit), B / 32));
}

void launch_mlp_tile_train(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, int act, uint32_t B, uint32_t dims, float loss_scale,
                           uint32_t loss_l2, const void* params16, const void* enc16, const float* target, const void* dout16, void* out16,
                           void* dldenc, int dldenc_pairs, float* wgrad_partial, float* loss_partial, void* wT) {
	TCNN_CHECK(B % 32 == 0, "tile train: batch must be a multiple of 32");
	TCNN_CHECK(tile_train_supported(W, IN, NH, 16, act), "tile train: unsupported shape");
	TCNN_CHECK(dout16 || dims <= 16, "tile train: at most 16 outputs");
	if (B == 0) return;
	TileTrainArgs a{};
	a.B = B;
	a.dims = dims;
	a.loss_l2 = loss_l2;
	a.loss_scale = loss_scale;
	a.n_total = (float)((uint64_t)B * dims);
	a.params = (const _Float16*)params16;
	const uint32_t ns = tile_train_n_streamed(W, IN, NH);
	if (ns) {
		TCNN_CHECK(wT != nullptr, "tile train: streamed hidden matrices need the transposed-weight buffer");
		const uint32_t n = ns * W * W;
		hipLaunchKernelGGL(k_tile_transpose_hidden, dim3((n + 255) / 256), dim3(256), 0, st, (const _Float16*)params16 + (size_t)W * IN,
		                   (_Float16*)wT, W, n);
	}
	a.wT = (const _Float16*)wT;
	a.enc = (const _Float16*)enc16;
	a.target = target;
	a.dout = (const _Float16*)dout16;
	a.out = (_Float16*)out16;
	a.dldenc = dldenc;
	a.dldenc_pairs = dldenc_pairs;
	a.wgrad_partial = wgrad_partial;
	a.loss_partial = loss_partial;
	const uint32_t blocks = tile_train_blocks(B, W, IN, NH);
	bool ok = false;
#define X(w, in, nh)                                                                                          \
	if (!ok && W == w && IN == in && NH == nh) {                                                              \
		ok = true;                                                                                            \
		if (act == ACT_RELU) {                                                                                \
			if (dout16) tile_launch<w, in, nh, Act::ReLU, true>(st, blocks, a);                                \
			else tile_launch<w, in, nh, Act::ReLU, false>(st, blocks, a);                                      \
		} else {                                                                                              \
			if (dout16) tile_launch<w, in, nh, Act::None, true>(st, blocks, a);                                \
			else tile_launch<w, in, nh, Act::None, false>(st, blocks, a);                                      \
		}                                                                                                     \
	}
	TILE_SHAPES(X)
#undef X
	TCNN_CHECK(ok, "tile train: shape not instantiated");
	TCNN_HIP_CHECK(hipGetLastError());
}

}  // namespace tcnn_amd
