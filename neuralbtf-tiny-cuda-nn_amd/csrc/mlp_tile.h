// mlp_tile.h -- fully fused MLP for every FullyFusedMLP shape the register-resident grid kernel
// (mlp_fused.h: W <= 64, grid input, two hidden layers) does not take: W in {16, 32, 64, 128}, any
// input encoding (hash grid, OneBlob, Identity) read as fp16 [B][IN], IN <= 128, 1..5 hidden layers,
// any output activation. Templates here; instantiated per width in mlp_tile_w{16,32,64,128}.hip.
//
// Reference: kernel_mlp_fused / kernel_mlp_fused_backward (fully_fused_mlp.cu:47-259, 499-557; widths
// 16/32/64/128 at :893-896) and the CUTLASS weight-gradient GEMMs (fully_fused_mlp.cu:735-836). The
// reference writes every hidden activation and every backprop temporary to HBM ([W x B] fp16 per
// layer, twice) and reads them back for the split-K weight gradients; for W128/H4 at B = 2^20 that is
// ~5 KB per sample.
//
// Training (k_mlp_tile_train): one workgroup owns the whole network for 32-sample tiles:
//   * all weights are staged once into LDS (W128/H4/IN32: 119 KB, padded rows, fp16);
//   * a tile's input and its NH post-activations stay in LDS ([32][W+8] fp16 per layer, 35 KB) for
//     the backward pass, the loss is fused after the output layer (with the output activation and
//     its transfer), and each backprop delta overwrites the activation slot it no longer needs;
//   * weight gradients accumulate in registers across all tiles the workgroup processes: wave w owns
//     output-row tiles w*W/64 .. of every matrix (the MFMA contracts over the 32 samples of a tile,
//     operands read from LDS with the gfx950 ds_read_b64_tr_b16 transpose read), so no cross-wave
//     reduction exists; one fp32 partial slab per workgroup leaves at the end;
//   * dL/d(encoding) = W0^T delta_1 leaves in the layout the grid backward reads (level-major
//     feature pairs) or AoS for the OneBlob / Identity input gradient.
// Inference (k_mlp_tile_infer, the reference's INFERENCE=true instantiation, :524-532): weight-
// stationary -- each wave keeps the A fragments of its two output-row tiles of every matrix in
// registers for the whole launch (no weight traffic after the first load), activations ping-pong
// between two LDS tiles, nothing but the input and the 16-wide output touches HBM.
// W16 networks run the W32 kernels on zero-padded weights: the padded neurons' pre-activations are
// exactly 0, their deltas exactly 0, so outputs and gradients equal the unpadded network's.
// fp32 MFMA accumulation (f32_16x16x32_f16), fp16 storage at the reference's points.
#pragma once

#include "kernels.h"
#include "mlp_fused.h"

namespace tcnn_amd {

constexpr int tile_kw(int WR) { return WR < 32 ? 32 : WR; }  // kernel width (W16 -> 32, zero-padded)
constexpr int tile_imax(int a, int b) { return a > b ? a : b; }
constexpr int tile_imin(int a, int b) { return a < b ? a : b; }

// ---------------------------------------------------------------------------------------------
// training
// ---------------------------------------------------------------------------------------------
// LDS halves of a tile workgroup of TS-sample tiles with the first NS hidden matrices streamed from L2
// instead of staged
constexpr int tile_rsw(int W) { return W + 8; }  // row stride of the W-wide LDS buffers (halves)
// (PP: one more [TS][RSW] slot, the backward's ping-pong delta buffer, tile_pp_ok)
constexpr int tile_halves(int W, int IN, int NH, int NS, int TS = 32, int PP = 0) {
	const int KP0 = (IN + 31) / 32 * 32, RS0 = KP0 + 8, RSW = tile_rsw(W), RSG = 24;
	return W * RS0 + (NH - 1 - NS) * W * RSW + 16 * RSW + TS * RS0 + (NH + PP) * TS * RSW + TS * RSG;
}
// waves per workgroup: W128 runs 8 (2 per SIMD, one 16-row tile of every matrix each) up to 4 hidden
// layers; with 5 its weight-gradient accumulators (>= 164 registers) spill at 256 registers per wave,
// so it runs 4 waves (1 per SIMD, 512 registers incl. AGPRs, two row tiles each); W64 4; W32 2 (one
// row tile each)
//
// Register-resident variant (RA): every hidden matrix's A fragments -- forward (the wave's output
// rows) and backward (the wave's input features, from the transposed copy) -- are loaded once per
// launch into registers and stay there; no hidden matrix is staged in LDS and no A operand is read
// from it. W64: 4 waves of one row tile each, two workgroups per CU (IN 128 with 5 hidden layers would
// spill at 256 registers). W128: 4 waves (one per SIMD, two row tiles each, up to 512 registers:
// 64 per hidden matrix for the fragments + the weight-gradient accumulators), for IN <= 32 and at most
// 3 hidden layers -- with 4 the kernel spills 24 registers and measured 2 % slower than the 8-wave
// LDS-staged kernel (profiles/r03_tile_ra_ab.json); measured 1.03-1.06x faster on the W64 configs and
// HashGrid + W128/H3.
constexpr bool tile_ra_ok(int W, int IN, int NH) {
	return NH > 1 && ((W == 64 && !(IN > 64 && NH > 4)) || (W == 128 && IN <= 32 && NH <= 3));
}
constexpr int tile_waves(int W, int NH, bool RA = false) { return W == 128 && NH < 5 && !RA ? 8 : (W == 32 ? 2 : 4); }
constexpr int tile_lds_limit() { return 160 * 1024; }
// fewest streamed hidden matrices that let the rest of the network + the tile's activations fit
// (RA: all of them, from registers)
constexpr int tile_n_streamed(int W, int IN, int NH, bool RA = false, int TS = 32, int PP = 0) {
	if (RA) return NH - 1;
	int ns = 0;
	while (ns < NH - 1 && tile_halves(W, IN, NH, ns, TS, PP) * 2 + tile_waves(W, NH) * 4 > tile_lds_limit()) ++ns;
	return ns;
}
// 64-sample tiles (TS = 64): half the workgroup barriers per sample (each layer's barrier now covers
// four 16-sample MFMA columns per row tile, the weight-gradient MFMAs contract over two 32-sample
// halves). For the 8-wave W128 kernel (enough waves for the output layer's four 16-sample columns),
// where at most one more hidden matrix has to move from LDS to L2 to make room for the larger tile
// (configs[3] HashGrid + W128/H4: 119 KB of staged weights + 38 KB of tile -> one hidden matrix read
// from L2, 158 KB; W128/H4 at IN 64: two instead of one, still 7 % faster with the streamed fragments
// loaded a layer ahead).
constexpr bool tile_ts64_ok(int W, int IN, int NH, bool RA) {
	return (!RA && W == 128 && tile_waves(W, NH) == 8 && tile_n_streamed(W, IN, NH, false, 64) <= tile_n_streamed(W, IN, NH, false, 32) + 1) ||
	       // register-resident kernels, 4 waves, nothing staged: W64 (IN 128 with 3+ hidden layers spills)
	       // and W128 (IN <= 32, <= 3 hidden layers)
	       (RA && W == 64 && tile_ra_ok(W, IN, NH) && (IN <= 64 || NH <= 2)) || (RA && W == 128 && tile_ra_ok(W, IN, NH));
}
// workgroups per CU the launch aims for: two waves per SIMD where the LDS (and, for W128 RA, the
// registers) allow
constexpr int tile_train_wg_per_cu(int W, int IN, int NH, bool RA = false, int TS = 32, int PP = 0) {
	return W == 128 && RA ? 1
	                      : tile_imax(1, tile_imin(8 / tile_waves(W, NH, RA),
	                                               tile_lds_limit() / (tile_halves(W, IN, NH, tile_n_streamed(W, IN, NH, RA, TS, PP), TS, PP) * 2 +
	                                                                   tile_waves(W, NH, RA) * 4)));
}
// Ping-pong delta buffer (PP): the backward writes delta_k into a spare [TS][RSW] slot or into a_NH's
// slot, alternating (delta_NH -> spare, delta_{NH-1} -> a_NH's slot, delta_{NH-2} -> spare, ...), so a
// delta never overwrites an operand another wave may still be reading and each backward layer needs
// one workgroup barrier instead of two (H4: 15 -> 11 per tile). Taken wherever the spare slot fits
// without streaming another hidden matrix or losing a workgroup per CU.
constexpr bool tile_pp_ok(int W, int IN, int NH, bool RA, int TS) {
	return tile_n_streamed(W, IN, NH, RA, TS, 1) == tile_n_streamed(W, IN, NH, RA, TS, 0) &&
	       tile_train_wg_per_cu(W, IN, NH, RA, TS, 1) == tile_train_wg_per_cu(W, IN, NH, RA, TS, 0) &&
	       tile_halves(W, IN, NH, tile_n_streamed(W, IN, NH, RA, TS, 1), TS, 1) * 2 + tile_waves(W, NH, RA) * 4 <= tile_lds_limit();
}

template <int WR, int IN, int NH, bool RA = false, int TS = 32>
struct TileLayout {
	static constexpr int W = tile_kw(WR);
	static_assert(W == 32 || W == 64 || W == 128, "tile engine: W in {16, 32, 64, 128}");
	static_assert(IN % 16 == 0 && IN <= 128, "tile engine: IN a multiple of 16, <= 128");
	static_assert(!RA || tile_ra_ok(W, IN, NH), "register-resident variant: shape out of its register budget");
	static constexpr int KP0 = (IN + 31) / 32 * 32;  // K of the first layer, padded to the MFMA depth
	// every LDS matrix (W0 and the input slot [.][RS0], the hidden matrices, Wout and the activation slots
	// [.][RSW]): rows padded by 16 B, and the 16-byte chunks of each pair swapped in rows 4..11 of every 16
	// (tile_ix) -- except W0 and the input slot of the 4-wave W128 kernel (5 hidden layers), whose
	// swizzled transposes cost 12 more spilled registers at its 512-register bound
	static constexpr bool SWZ = true, SWZ0 = !(W == 128 && tile_waves(W, NH, RA) == 4);
	static constexpr int RS0 = KP0 + 8, RSW = tile_rsw(W), RSG = 24;
	static constexpr int WAVES = tile_waves(W, NH, RA), NTHR = WAVES * 64;
	static constexpr int MT = W / 16, MTW = MT / WAVES;  // output-row tiles per matrix / per wave
	static constexpr int KT0 = IN / 16;              // feature tiles of the input
	// hidden matrices 1..NS are not staged: their forward A fragments come from the fp16 parameters
	// (L2-resident, every workgroup reads the same 32 KB), their backward ones from a transposed copy
	// (RA: loaded once into registers)
	static constexpr int PP = tile_pp_ok(W, IN, NH, RA, TS) ? 1 : 0;
	static constexpr int NS = tile_n_streamed(W, IN, NH, RA, TS, PP);
	static constexpr int NTAU = TS / 16, KH = TS / 32;  // 16-sample MFMA columns / 32-sample K halves per tile
	static_assert(TS == 32 || (TS == 64 && tile_ts64_ok(W, IN, NH, RA)), "tile samples: 32, or 64 where tile_ts64_ok");
	static_assert(NTAU <= WAVES, "one wave per 16-sample column of the output layer");
	static_assert(NS == 0 || W == WR, "streamed matrices only for unpadded widths");
	static constexpr int oW0 = 0, oWh = oW0 + W * RS0, oWo = oWh + (NH - 1 - NS) * W * RSW;
	static constexpr int oX = oWo + 16 * RSW;                 // slot 0: the tile's input [TS][RS0]
	static constexpr int oA = oX + TS * RS0;                  // slots 1..NH: [TS][RSW]
	static constexpr int oG = oA + NH * TS * RSW;             // dL/dy of the tile [TS][RSG]
	static constexpr int oD = oG + TS * RSG;                  // PP: the spare delta slot [TS][RSW]
	static constexpr int HALVES = oD + PP * TS * RSW;
	static constexpr int BYTES = HALVES * 2 + WAVES * 4;       // + per-wave loss
	static constexpr int N_MLP = WR * IN + (NH - 1) * WR * WR + 16 * WR;  // parameters (unpadded)
	static constexpr int WG_PER_CU = tile_train_wg_per_cu(W, IN, NH, RA, TS, PP);
	// waves per SIMD the launch runs (amdgpu_waves_per_eu: caps the registers so they fit)
	static constexpr int WAVES_PER_EU = tile_imax(1, WG_PER_CU * WAVES / 4);
	static_assert(HALVES == tile_halves(W, IN, NH, NS, TS, PP), "layout");
	static_assert(oWh % 8 == 0 && oWo % 8 == 0 && oX % 8 == 0 && oA % 8 == 0 && oG % 8 == 0 && oD % 8 == 0, "16-byte alignment");
	static_assert(BYTES <= tile_lds_limit(), "tile exceeds the LDS");
};

// Tile LDS swizzle: in rows r with r % 16 in 4..11 the two 16-byte chunks of every 32-byte pair trade
// places (chunk c -> c ^ 1). Chunk bit 0 comes from the lane in every access of the kernel (row-fragment
// ds_read_b128: q & 1; ds_read_b64_tr_b16: (c >> 1) & 1; h4 loads / stores: q >> 1), so the swap stays a
// per-lane constant and every compile-time offset remains an immediate. Searched over all per-row
// bit-0 swaps against the kernel's access patterns (64-wide banking of ds_read_b128 in its 4 x 16 lane
// groups and of ds_read_b64[_tr_b16] in 2 x 32, 32-wide of ds_write_b64 in 4 x 16) at the 272-byte row
// stride: the row-fragment reads become conflict-free (2-way before: lanes c = 11, q = 1 and c = 12,
// q = 0 met on one slot), transpose reads and stores stay 2-way, h4 loads go 1 -> 2-way; weighted by
// the configs[3] kernel's instruction mix, 23 % fewer LDS cycles. (A full chunk XOR makes the
// transpose reads conflict-free too, but its per-access offsets are lane-dependent XORs the compiler
// keeps in registers: 50-140 spills at 256 VGPRs.)
__device__ __forceinline__ int tile_swz(int r) { return (((r & 15) + 4) >> 3) & 1; }
template <bool SWZ, int RS>
__device__ __forceinline__ int tile_ix(int row, int col) {
	if constexpr (SWZ) return row * RS + (col ^ (tile_swz(row) << 3));
	else return row * RS + col;
}
// the same with the column split into a part that is a multiple of 16 (compile-time / wave-uniform) and
// the lane's part (< 16, holding bit 3): the swap touches only the lane's part, so the compiler keeps one
// per-lane base and folds the rest into immediate offsets
template <bool SWZ, int RS>
__device__ __forceinline__ int tile_ix(int row, int col16, int col_lane) {
	if constexpr (SWZ) return row * RS + col16 + (col_lane ^ (tile_swz(row) << 3));
	else return row * RS + col16 + col_lane;
}
struct TileTrainArgs {
	uint32_t B, dims, loss_l2;
	float loss_scale, n_total;
	int out_act;             // output activation (ACT_*), applied after the output layer, transfer before the backward
	const _Float16* params;  // [W0 | hidden | Wout] fp16 (unpadded width WR)
	const _Float16* wT;      // streamed hidden matrices 1..NS transposed, [NS][W (in)][W (out)] fp16
	const _Float16* enc;     // encoded input fp16 [B][IN]
	const float* target;     // [B][dims] (loss)
	const _Float16* dout;    // external dL/d(output) fp16 [B][16] (loss-scaled by the caller; nullptr: the loss)
	_Float16* out;           // optional network output fp16 [B][16]
	void* dldenc;            // optional dL/d(encoding): pairs [IN/2][B] (uint32) or AoS fp16 [B][IN]
	int dldenc_pairs;
	float* wgrad_partial;    // [gridDim.x][N_MLP]
	float* loss_partial;     // [gridDim.x]
	// GENC kernels (the grid encoding gathered in-kernel instead of read from `enc`, r06): positions
	// fp32 [B][2], the fp16 grid table as half2 entries, the level table, the hash-grid flag, and whether
	// the branch-free in-range index applies (GridEncodingHost::inrange_index_ok)
	const float* gpos;
	const uint32_t* gtable;
	const LevelInfo* glevels;
	uint32_t ghash, ginrange;
};

// LDS beyond the layout that the in-kernel grid encode (GENC) uses: the level table (16 B per level)
// and one 64-byte position buffer per wave (8 samples x 2 dimensions)
constexpr int tile_genc_extra_bytes(int IN, int WAVES) { return (IN / 2) * 16 + WAVES * 64; }
constexpr int tile_genc_base_bytes(int bytes) { return (bytes + 15) / 16 * 16; }

__device__ __forceinline__ h8 zero8() { return h8{0, 0, 0, 0, 0, 0, 0, 0}; }

template <Act ACT>
__device__ __forceinline__ h4 tile_act(f4 v) {
	return act_fwd<ACT>(v);
}

// output activation on the fp32 accumulator, rounded once (the layer-wise engine's order)
__device__ __forceinline__ h4 out_act_fwd(int a, f4 y) {
	if (a == ACT_NONE) return __builtin_convertvector(y, h4);
	h4 r;
#pragma unroll
	for (int k = 0; k < 4; ++k) r[k] = f16_rn(act_fwd_ool(a, y[k]));
	return r;
}

// launch bounds as plain function calls (a template-id's commas would split the macro arguments)
constexpr int tile_train_nthr(int WR, int NH, bool RA) { return tile_waves(tile_kw(WR), NH, RA) * 64; }
constexpr int tile_train_weu(int WR, int IN, int NH, bool RA, int TS) {
	return tile_imax(1, tile_train_wg_per_cu(tile_kw(WR), IN, NH, RA, TS, tile_pp_ok(tile_kw(WR), IN, NH, RA, TS) ? 1 : 0) *
	                        tile_waves(tile_kw(WR), NH, RA) / 4);
}

// GENC = 0: the tile's input rows come from a.enc (AoS fp16 [B][IN]). GENC = 1 + (int)HashType: the
// 2-D, 2-feature grid encoding is gathered in the kernel (r06, VERDICT r05 item 3: configs[3]'s separate
// 122 us AoS encode pass and its 64 MB write + re-read go away). The gathers of tile t+1 are issued as
// LDS-DMA (global_load_lds_dword: no registers held) into a slot the backward of tile t no longer needs,
// two backward layers before the tile ends, so their latency runs under those layers' MFMAs; at the
// start of tile t+1 each lane combines its 2 levels x 4 corners with the weights (the fp16 FMA chain of
// encode_level_f2 / _inrange, bit-identical) into slot 0. Every staging buffer is wave-local: a wave
// waits only on its own DMA (vmcnt) before reading it back. The tile's positions arrive the same way
// one tile ahead. Shape: 8 waves, 64-sample tiles, IN = 32 (16 levels: lane = 8 samples x 8 level pairs).
template <int WR, int IN, int NH, Act ACT, bool RA, int TS, int GENC = 0>
__global__ __launch_bounds__(tile_train_nthr(WR, NH, RA), tile_train_weu(WR, IN, NH, RA, TS)) void k_mlp_tile_train(const TileTrainArgs a) {
	using L = TileLayout<WR, IN, NH, RA, TS>;
	constexpr int W = L::W, NTAU = L::NTAU, KH = L::KH;
	constexpr int MTW = L::MTW, KT0 = L::KT0, RS0 = L::RS0, RSW = L::RSW, RSG = L::RSG;
	constexpr int WAVES = L::WAVES, NTHR = L::NTHR;
	constexpr int NTW = L::MT / WAVES;  // Wout column tiles per wave (= MTW)
	constexpr bool SWZ = L::SWZ, SWZ0 = L::SWZ0;
	extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
	const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	const int c = lane & 15, q = lane >> 4;
	// The lane's part of every LDS address, computed once (with the W128 swizzle, tile_ix): the accesses
	// below add only compile-time / wave-uniform offsets, which the compiler folds into the instructions'
	// immediate offsets instead of keeping one address register per access.
	//   row fragment (ds_read_b128): row 16 k + c, columns 32 s + 8 q ..+7    -> lf + 16 k RS + 32 s
	//   h4 (ds_read_b64 / ds_write_b64): row 16 k + c, columns 16 t + 4 q ..+3 -> l4 + 16 k RS + 16 t
	//   transpose read (trw / trwo / trx): rows 8 q + (c >> 2) and + 4, columns 16 t + 4 (c & 3) ..+3
	const int lf = tile_ix<SWZ, RSW>(c, 0, 8 * q), l4 = tile_ix<SWZ, RSW>(c, 0, 4 * q), lf0 = tile_ix<SWZ0, RS0>(c, 0, 8 * q);
	const int ltx = tile_ix<SWZ0, RS0>(8 * q + (c >> 2), 0, 4 * (c & 3)), ltx4 = tile_ix<SWZ0, RS0>(8 * q + (c >> 2) + 4, 0, 4 * (c & 3));
	const int ltr = tile_ix<SWZ, RSW>(8 * q + (c >> 2), 0, 4 * (c & 3)), ltr4 = tile_ix<SWZ, RSW>(8 * q + (c >> 2) + 4, 0, 4 * (c & 3));
	const int lto = tile_ix<SWZ, RSW>(8 * (q & 1) + (c >> 2), 0, 4 * (c & 3)), lto4 = tile_ix<SWZ, RSW>(8 * (q & 1) + (c >> 2) + 4, 0, 4 * (c & 3));
	auto ixf = [&](bool x0, int row16, int col32) { return x0 ? row16 * RS0 + col32 + lf0 : row16 * RSW + col32 + lf; };
	auto ix4 = [&](int row16, int col16) { return row16 * RSW + col16 + l4; };
	auto trpair = [](const _Float16* lo, const _Float16* hi) {
		typedef __attribute__((address_space(3))) s4 lds_s4;
		const s4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)lo);
		const s4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)hi);
		return cat8(__builtin_bit_cast(h4, a), __builtin_bit_cast(h4, b));
	};
	// S[8q + e][16 t + c] of a W-wide buffer (Wout: the rows 8 (q & 1) + e of its 16)
	auto trw = [&](const _Float16* S, int t) { return trpair(S + ltr + 16 * t, S + ltr4 + 16 * t); };
	auto trwo = [&](const _Float16* S, int t) { return trpair(S + lto + 16 * t, S + lto4 + 16 * t); };
	// Sample-indexed transposes (the weight-gradient operands: rows are the tile's samples, the MFMA's K):
	// the lo read takes the even rows 8 q + 2 j and the hi read the odd ones (j = c >> 2), so each 32-lane
	// half reads 8 rows two apart -- conflict-free at every row stride (rows four apart, as in trw, put two
	// rows' 32-byte segments on overlapping banks: 2-way). K index 8 q + e then holds sample 8 q + 2 e
	// (lo) / 8 q + 2 e + 1 (hi) in both operands of an MFMA, a permutation of its sum, so every
	// weight-gradient MFMA reads both operands this way. (Not in the 4-wave W128 kernel: at its
	// 512-register bound the extra lane offsets cost 13 spilled registers; it keeps rows four apart.)
	const int lts = SWZ0 ? tile_ix<SWZ, RSW>(8 * q + 2 * (c >> 2), 0, 4 * (c & 3)) : 0;
	const int lts1 = SWZ0 ? tile_ix<SWZ, RSW>(8 * q + 2 * (c >> 2) + 1, 0, 4 * (c & 3)) : 0;
	const int ltsx = SWZ0 ? tile_ix<SWZ0, RS0>(8 * q + 2 * (c >> 2), 0, 4 * (c & 3)) : 0;
	const int ltsx1 = SWZ0 ? tile_ix<SWZ0, RS0>(8 * q + 2 * (c >> 2) + 1, 0, 4 * (c & 3)) : 0;
	const int ltsg = SWZ0 ? (8 * q + 2 * (c >> 2)) * RSG + 4 * (c & 3) : 0;
	auto trs = [&](const _Float16* S, int t) { return trpair(S + lts + 16 * t, S + lts1 + 16 * t); };
	auto trsx = [&](const _Float16* S, int t) { return trpair(S + ltsx + 16 * t, S + ltsx1 + 16 * t); };
	auto trsg = [&](const _Float16* S) { return trpair(S + ltsg, S + ltsg + RSG); };
	auto trx = [&](const _Float16* S, int t) {  // [.][RS0] buffers
		if constexpr (SWZ0) return trpair(S + ltx + 16 * t, S + ltx4 + 16 * t);
		else return lds_trfrag(S, RS0, q, c, t);
	};
	const f4 fz = {0.0f, 0.0f, 0.0f, 0.0f};
	float* wloss = (float*)(smem + L::HALVES);
	const bool ext = a.dout != nullptr;
	// OP: the output rows are stored transposed 4 x 4 (out_row, mlp_fused.h), so lane group q holds
	// output 4r + q in register r and the loss of a <= 4-output network runs once per lane instead of
	// once per r (waves 0, 1 compute it while the other waves wait at the next barrier). Not for the
	// W128 / >= 4 hidden-layer kernels, which sit at their 256-register bound and spill with it.
	constexpr bool OP = !(W >= 128 && NH >= 4);

	// ---- weights -> LDS (rows padded; first-layer columns [IN, KP0) and W16's padded neurons zero) ----
	{
		const _Float16* p = a.params;
		for (int idx = tid; idx < W * (L::KP0 / 8); idx += NTHR) {
			const int r = idx / (L::KP0 / 8), c8 = idx % (L::KP0 / 8);
			*(h8*)(smem + L::oW0 + tile_ix<SWZ0, RS0>(r, 8 * c8)) = (r < WR && 8 * c8 < IN) ? *(const h8*)(p + (size_t)r * IN + 8 * c8) : zero8();
		}
		p += WR * IN;
		for (int idx = tid; idx < (NH - 1 - L::NS) * W * (W / 8); idx += NTHR) {
			const int r = idx / (W / 8), c8 = idx % (W / 8);  // r over the staged hidden rows
			const int j = r / W + L::NS, rr = r % W;
			*(h8*)(smem + L::oWh + (r / W) * W * RSW + tile_ix<SWZ, RSW>(rr, 8 * c8)) =
			    (rr < WR && 8 * c8 < WR) ? *(const h8*)(p + ((size_t)j * WR + rr) * WR + 8 * c8) : zero8();
		}
		p += (NH - 1) * WR * WR;
		for (int idx = tid; idx < 16 * (W / 8); idx += NTHR) {
			const int r = idx / (W / 8), c8 = idx % (W / 8);
			*(h8*)(smem + L::oWo + tile_ix<SWZ, RSW>(OP ? out_row(r) : r, 8 * c8)) = 8 * c8 < WR ? *(const h8*)(p + (size_t)r * WR + 8 * c8) : zero8();
		}
		// zero the padded input columns of slot 0 once (the input loads never write them)
		if (L::KP0 > IN)
			for (int idx = tid; idx < TS * (L::KP0 - IN); idx += NTHR)
				smem[L::oX + tile_ix<SWZ0, RS0>(idx / (L::KP0 - IN), IN + idx % (L::KP0 - IN))] = (_Float16)0.0f;
	}
	// staged matrices (m == 0 or m > NS); streamed ones (1 <= m <= NS) are read from global memory
	auto Wm = [&](int m) -> const _Float16* { return m == 0 ? smem + L::oW0 : smem + L::oWh + (m - 1 - L::NS) * W * RSW; };
	auto streamed = [](int m) { return m >= 1 && m <= L::NS; };
	auto slot = [&](int m) -> _Float16* { return m == 0 ? smem + L::oX : smem + L::oA + (m - 1) * TS * RSW; };
	// where delta_k lives: PP -- the spare slot for even NH - k, a_NH's slot for odd; otherwise a_k's slot
	auto dslot = [&](int k) -> _Float16* { return L::PP ? ((NH - k) % 2 == 0 ? smem + L::oD : slot(NH)) : slot(k); };
	_Float16* sG = smem + L::oG;

	// ---- register accumulators of this wave's weight-gradient rows ----
	f4 dW0[MTW][KT0];
	f4 dWh[NH > 1 ? NH - 1 : 1][MTW][L::MT];
	f4 dWo[NTW];
	// RA: the hidden matrices' forward / backward A fragments, loaded once (rows resp. input features
	// 16 (wave MTW + i) + c, K columns 32 s + 8 q ..+7)
	constexpr int NRA = RA ? NH - 1 : 1;
	h8 pag[NRA][MTW][W / 32], pagT[NRA][MTW][W / 32];
	if constexpr (RA) {
#pragma unroll
		for (int j = 0; j < NH - 1; ++j)
#pragma unroll
			for (int i = 0; i < MTW; ++i)
#pragma unroll
				for (int s = 0; s < W / 32; ++s) {
					const size_t o = (size_t)j * W * W + (size_t)(16 * (wave * MTW + i) + c) * W + 32 * s + 8 * q;
					pag[j][i][s] = *(const h8*)(a.params + (size_t)W * IN + o);
					pagT[j][i][s] = *(const h8*)(a.wT + o);
				}
	}
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
	constexpr int XV = TS * IN / 8, XPT = GENC ? 1 : (XV + NTHR - 1) / NTHR;
	const uint32_t n_tiles = a.B / TS;
	uint32_t tile = blockIdx.x;
	h8 xr[XPT];
	auto load_x = [&](uint32_t t) {
#pragma unroll
		for (int j = 0; j < XPT; ++j) {
			const int idx = tid + NTHR * j;
			if (idx < XV) xr[j] = *(const h8*)(a.enc + ((size_t)t * TS + idx / (IN / 8)) * IN + 8 * (idx % (IN / 8)));
		}
	};

	// ---- in-kernel grid encode (GENC) ----
	static_assert(!GENC || (TS == 64 && WAVES == 8 && IN == 32 && !L::PP && NH >= 2), "GENC: the 8-wave W128 kernel, IN 32, no ping-pong slot");
	constexpr HashType GH = (HashType)(GENC > 0 ? GENC - 1 : 0);
	const int wave_s = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform offsets stay in SGPRs
	LevelInfo* gLvl = (LevelInfo*)((char*)smem + tile_genc_base_bytes(L::BYTES));
	float* gPos = (float*)((char*)gLvl + (IN / 2) * 16) + wave_s * 16;  // this wave's 8 samples x 2 dims
	// staging of the wave's 8 gathers per lane ([k][corner][lane] dwords): slot NH, dead from the start of
	// the backward's layer NH - 2 to the end of the tile (its delta_NH was last read by layer NH - 1)
	uint32_t* gStage = (uint32_t*)(smem + L::oA + (NH - 1) * TS * RSW) + wave_s * 8 * 64;
	// The LDS-DMA loads: lds_dma.h (inline asm; the waits are ours -- each reader of a buffer waits for its
	// own wave's DMA first)
	auto lds_dma = [](const void* g, const void* l) { lds_dma_u32(g, l); };
	auto genc_pos_dma = [&](uint32_t t) {  // positions of tile t's samples 8 wave .. +7 -> gPos (lanes 0..15)
		if (lane < 16) lds_dma(a.gpos + ((size_t)t * TS + 8 * wave_s) * 2 + lane, gPos);
	};
	auto genc_issue = [&]() {  // corner gathers of the tile whose positions are in gPos -> gStage
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's position DMA landed
		const int sl = lane >> 3, j = lane & 7;
		const float x0 = gPos[2 * sl], x1 = gPos[2 * sl + 1];
		const bool inr = x0 >= 0.0f && x0 <= 1.0f && x1 >= 0.0f && x1 <= 1.0f;
		const bool fast = a.ginrange && __builtin_amdgcn_ballot_w64(!inr) == 0;
#pragma unroll
		for (int k = 0; k < 2; ++k) {
			const LevelInfo li = gLvl[2 * j + k];
			float pos[2];
			uint32_t pg[2];
			pos_fract(x0, li.scale, Interp::Linear, pos[0], pg[0]);
			pos_fract(x1, li.scale, Interp::Linear, pos[1], pg[1]);
			uint32_t idx[4];
			if (fast) {  // grid_index_inrange's arithmetic (encode_level_f2_inrange)
				const LevelConsts<2> lc = level_consts<2>(li, a.ghash != 0);
#pragma unroll
				for (int cc = 0; cc < 4; ++cc) {
					uint32_t h = 0, dn = 0;
#pragma unroll
					for (int d = 0; d < 2; ++d) {
						const uint32_t bb = (cc >> d) & 1u;
						h ^= (pg[d] + bb) * hash_prime<GH>(d);
						dn += (pg[d] + bb) * lc.sd[d];
					}
					const uint32_t dm = __builtin_elementwise_min(dn, dn - lc.size);
					idx[cc] = li.offset + (((h & lc.hmask) & lc.m) | (dm & ~lc.m));
				}
			} else {
#pragma unroll
				for (int cc = 0; cc < 4; ++cc) {
					uint32_t local[2] = {pg[0] + (cc & 1u), pg[1] + ((cc >> 1) & 1u)};
					idx[cc] = li.offset + grid_index<2, GH>(a.ghash != 0, li.size, li.res, local);
				}
			}
#pragma unroll
			for (int cc = 0; cc < 4; ++cc)
				lds_dma(a.gtable + idx[cc], gStage + (4 * k + cc) * 64);
		}
	};
	auto genc_finish = [&](bool first) {  // gStage + gPos -> this wave's 8 samples x 16 levels of slot 0
		// this wave's gathers landed. vmcnt(0), not vmcnt(the stores issued after them): loads and stores
		// share the counter but need not complete in order with each other -- a count that skipped the
		// previous tile's dL/d(encoding) stores read stale staging (r06, the same wait in the fused
		// kernel's prefetch experiment: non-deterministic results at 2^18 points)
		(void)first;
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		const int sl = lane >> 3, j = lane & 7;
		const float x0 = gPos[2 * sl], x1 = gPos[2 * sl + 1];
#pragma unroll
		for (int k = 0; k < 2; ++k) {
			const int level = 2 * j + k;
			const float sc = gLvl[level].scale;
			float pos[2];
			uint32_t pg[2];
			pos_fract(x0, sc, Interp::Linear, pos[0], pg[0]);
			pos_fract(x1, sc, Interp::Linear, pos[1], pg[1]);
			float wf[4];
			_Float16 w16[4];
#pragma unroll
			for (int cc = 0; cc < 4; ++cc) {
				float w = 1.0f;
#pragma unroll
				for (int d = 0; d < 2; ++d) w *= ((cc >> d) & 1) ? pos[d] : 1.0f - pos[d];
				wf[cc] = w;
			}
			f16_rn_pairs(wf, w16);
			h2 r = {(_Float16)0.0f, (_Float16)0.0f};
#pragma unroll
			for (int cc = 0; cc < 4; ++cc) {
				const h2 wv = {w16[cc], w16[cc]};
				r = pk_fma_f16(wv, __builtin_bit_cast(h2, gStage[(4 * k + cc) * 64 + lane]), r);
			}
			*(h2*)(slot(0) + tile_ix<SWZ0, RS0>(8 * wave_s + sl, 2 * level)) = r;
		}
	};
	if constexpr (GENC) {
		for (int l = tid; l < IN / 2; l += NTHR) gLvl[l] = a.glevels[l];
		__syncthreads();
		if (tile < n_tiles) {
			genc_pos_dma(tile);
			genc_issue();
		}
	} else {
		if (tile < n_tiles) load_x(tile);
	}
	__syncthreads();

	for (; tile < n_tiles; tile += gridDim.x) {
		const uint32_t base = tile * TS;
		// ---- input tile -> slot 0; prefetch the next tile's rows (GENC: positions) ----
		if constexpr (GENC) {
			genc_finish(tile == blockIdx.x);  // the first tile has no stores issued after its gathers
			if (tile + gridDim.x < n_tiles) genc_pos_dma(tile + gridDim.x);  // gPos read above (data-dependent) first
		} else {
#pragma unroll
			for (int j = 0; j < XPT; ++j) {
				const int idx = tid + NTHR * j;
				if (idx < XV) *(h8*)(slot(0) + tile_ix<SWZ0, RS0>(idx / (IN / 8), 8 * (idx % (IN / 8)))) = xr[j];
			}
			if (tile + gridDim.x < n_tiles) load_x(tile + gridDim.x);
		}

		// targets / external dL/dy of this wave's output lanes (waves 0 .. NTAU-1: 16-sample column tau = wave)
		// (the external dL/dy's h4 rides in tg[0..1]: the two cases exclude each other, 2 registers saved)
		float tg[4] = {0.0f, 0.0f, 0.0f, 0.0f};
		typedef float tile_f2 __attribute__((ext_vector_type(2)));
		if (wave < NTAU) {
			const uint32_t i = base + 16 * wave + c;
			if (ext) {
				h4 gext;
				if constexpr (OP) {
					const _Float16* dp = a.dout + (size_t)i * 16 + q;
					gext = h4{dp[0], dp[4], dp[8], dp[12]};
				} else {
					gext = *(const h4*)(a.dout + (size_t)i * 16 + 4 * q);
				}
				const tile_f2 gb2 = __builtin_bit_cast(tile_f2, gext);
				tg[0] = gb2[0], tg[1] = gb2[1];
			} else if constexpr (OP) {  // register 0 only: outputs 4.. of a wider network are read in the loss
				if (q < (int)a.dims) tg[0] = a.target[(size_t)i * a.dims + q];
			} else {
#pragma unroll
				for (int r = 0; r < 4; ++r)
					if (4 * q + r < (int)a.dims) tg[r] = a.target[(size_t)i * a.dims + 4 * q + r];
			}
		}
		// streamed hidden matrices: each layer's A fragments are loaded one layer ahead (the first one
		// before this barrier), so their L2 latency runs under the previous layer instead of in front of
		// this layer's MFMAs (all waves of the workgroup reach a layer together: nothing else hides it)
		auto load_ag = [&](int m, h8 (&dst)[MTW][W / 32]) {
			const _Float16* Wg = a.params + (size_t)W * IN + (size_t)(m - 1) * W * W;
#pragma unroll
			for (int i = 0; i < MTW; ++i)
#pragma unroll
				for (int s = 0; s < W / 32; ++s) dst[i][s] = *(const h8*)(Wg + (size_t)(16 * (wave * MTW + i) + c) * W + 32 * s + 8 * q);
		};
		h8 agn[MTW][W / 32];
		if (!RA && NH > 1 && streamed(1)) load_ag(1, agn);
		__syncthreads();

		// ---- forward: a_{m+1} = act(M_m a_m), this wave's output-row tiles ----
#pragma unroll
		for (int m = 0; m < NH; ++m) {
			const int KS = (m == 0 ? L::KP0 : W) / 32;
			const _Float16* Wt = streamed(m) ? nullptr : Wm(m);
			const _Float16* in = slot(m);
			f4 acc[MTW][NTAU];
#pragma unroll
			for (int i = 0; i < MTW; ++i)
#pragma unroll
				for (int tau = 0; tau < NTAU; ++tau) acc[i][tau] = fz;
			h8 ag[MTW][W / 32];  // a streamed layer's A fragments, all loads issued before the first MFMA
			if (RA && streamed(m)) {
#pragma unroll
				for (int i = 0; i < MTW; ++i)
#pragma unroll
					for (int s = 0; s < W / 32; ++s) ag[i][s] = pag[m >= 1 ? m - 1 : 0][i][s];
			} else if (streamed(m)) {
#pragma unroll
				for (int i = 0; i < MTW; ++i)
#pragma unroll
					for (int s = 0; s < W / 32; ++s) ag[i][s] = agn[i][s];
				if (m + 1 < NH && streamed(m + 1)) load_ag(m + 1, agn);
			}
#pragma unroll
			for (int s = 0; s < KS; ++s) {
				h8 b[NTAU];
#pragma unroll
				for (int tau = 0; tau < NTAU; ++tau) b[tau] = *(const h8*)(in + ixf(m == 0, 16 * tau, 32 * s));
#pragma unroll
				for (int i = 0; i < MTW; ++i) {
					const h8 af = streamed(m) ? ag[i][s] : *(const h8*)(Wt + ixf(m == 0, 16 * (wave * MTW + i), 32 * s));
#pragma unroll
					for (int tau = 0; tau < NTAU; ++tau) acc[i][tau] = mfma16(af, b[tau], acc[i][tau]);
				}
			}
			_Float16* outs = slot(m + 1);
#pragma unroll
			for (int i = 0; i < MTW; ++i)
#pragma unroll
				for (int tau = 0; tau < NTAU; ++tau)
					*(h4*)(outs + ix4(16 * tau, 16 * (wave * MTW + i))) = tile_act<ACT>(acc[i][tau]);
			__syncthreads();
		}

		// ---- output layer (+ output activation) + loss + output transfer (waves 0 .. NTAU-1: tau = wave) ----
		if (wave < NTAU) {
			const int tau = wave;
			const _Float16* aN = slot(NH);
			f4 y = fz;
#pragma unroll
			for (int s = 0; s < W / 32; ++s)
				y = mfma16(*(const h8*)(smem + L::oWo + ixf(false, 0, 32 * s)), *(const h8*)(aN + ixf(false, 16 * tau, 32 * s)), y);
			const uint32_t i = base + 16 * tau + c;
			const h4 yh = out_act_fwd(a.out_act, y);
			if (a.out) {
				if constexpr (OP) {
#pragma unroll
					for (int r = 0; r < 4; ++r) a.out[(size_t)i * 16 + 4 * r + q] = yh[r];
				} else {
					*(h4*)(a.out + (size_t)i * 16 + 4 * q) = yh;
				}
			}
			h4 g = zero4();
			if (ext) {
				g = __builtin_bit_cast(h4, tile_f2{tg[0], tg[1]});
			} else {
#pragma unroll
				for (int r = 0; r < 4; ++r) {
					if (OP && 4u * r >= a.dims) break;  // wave-uniform: r = 0 only for <= 4 outputs
					const uint32_t o = OP ? 4 * r + q : 4 * q + r;
					if (o < a.dims) {
						const float p = (float)yh[r];
						const float pse = a.loss_l2 ? 1.0f : __builtin_fmaf(p, p, 0.01f);  // relative_l2.h:67-75 / l2.h:66-74
						const float t = (!OP || r == 0) ? tg[r] : a.target[(size_t)(base + 16 * tau + c) * a.dims + o];
						const float d = p - t;
						loss += d * d / pse / a.n_total;
						g[r] = f16_rn(a.loss_scale * (2.0f * d / pse) / a.n_total);
					}
				}
			}
			// output-activation transfer given the output (fully_fused_mlp.cu:759-762)
			if (a.out_act != ACT_NONE) {
#pragma unroll
				for (int r = 0; r < 4; ++r) g[r] = f16_rn(act_bwd_ool(a.out_act, (float)g[r], (float)yh[r]));
			}
			*(h4*)(sG + (16 * tau + c) * RSG + 4 * q) = g;
		}
		__syncthreads();

		// a streamed matrix's transposed A fragments (A[feature][neuron] = M^T rows of this wave's tiles)
		// for the backward, loaded one layer ahead like the forward's -- not in the 4-wave W128 kernel, where
		// the 32 extra registers spill at its 512-register bound
		constexpr bool PFB = !RA && SWZ0;
		auto load_agT = [&](int m, h8 (&dst)[MTW][W / 32]) {
			const _Float16* WgT = a.wT + (size_t)(m - 1) * W * W;
#pragma unroll
			for (int i = 0; i < MTW; ++i)
#pragma unroll
				for (int s = 0; s < W / 32; ++s) dst[i][s] = *(const h8*)(WgT + (size_t)(16 * (wave * MTW + i) + c) * W + 32 * s + 8 * q);
		};
		h8 agTn[MTW][W / 32];
		if (PFB && NH > 1 && streamed(NH - 1)) load_agT(NH - 1, agTn);
		// ---- dWout += G^T a_NH ; delta_NH = act'(a_NH) * (Wout^T G) ----
		h4 dl[MTW][NTAU];
		{
			const _Float16* aN = slot(NH);
#pragma unroll
			for (int kh = 0; kh < KH; ++kh) {
				if constexpr (SWZ0) {
					const h8 ga = trsg(sG + 32 * kh * RSG);  // A[out c][sample 32kh+8q+e] (even/odd rows)
#pragma unroll
					for (int i = 0; i < NTW; ++i) dWo[i] = mfma16(ga, trs(aN + 32 * kh * RSW, wave * NTW + i), dWo[i]);
				} else {
					const h8 ga = lds_trfrag(sG + 32 * kh * RSG, RSG, q, c, 0);  // A[out c][sample 32kh+8q+e]
#pragma unroll
					for (int i = 0; i < NTW; ++i) dWo[i] = mfma16(ga, trw(aN + 32 * kh * RSW, wave * NTW + i), dWo[i]);
				}
			}
			h8 gb[NTAU];
#pragma unroll
			for (int tau = 0; tau < NTAU; ++tau) gb[tau] = q < 2 ? *(const h8*)(sG + (16 * tau + c) * RSG + 8 * q) : zero8();
#pragma unroll
			for (int i = 0; i < MTW; ++i) {
				const int mt = wave * MTW + i;
				// A[neuron][out 8q+e]: K = 16 outputs, the upper half of the MFMA depth is zero through gb.
				// Every lane takes part in the transpose read (lanes q >= 2 re-read rows 0..15): the
				// ds_read_b64_tr_b16 exchange under a partial EXEC mask returned garbage (NaN deltas).
				const h8 af = trwo(smem + L::oWo, mt);
#pragma unroll
				for (int tau = 0; tau < NTAU; ++tau) {
					const f4 v = mfma16(af, gb[tau], fz);
					dl[i][tau] = act_bwd<ACT>(*(const h4*)(aN + ix4(16 * tau, 16 * mt)), v);
				}
			}
		}
		if constexpr (!L::PP) __syncthreads();  // a_NH is read above by every wave
		{
			_Float16* dN = dslot(NH);
#pragma unroll
			for (int i = 0; i < MTW; ++i)
#pragma unroll
				for (int tau = 0; tau < NTAU; ++tau) *(h4*)(dN + ix4(16 * tau, 16 * (wave * MTW + i))) = dl[i][tau];
		}
		__syncthreads();

		// ---- hidden layers and the first layer, last to first ----
#pragma unroll
		for (int m = NH - 1; m >= 0; --m) {
			if constexpr (GENC) {  // slot NH is dead from here on: the next tile's gathers go there
				if (m == NH - 2 && tile + gridDim.x < n_tiles) genc_issue();
			}
			const _Float16* dsl = dslot(m + 1);  // delta_{m+1} [sample][neuron]
			const _Float16* am = slot(m);       // a_m [sample][feature]
			const int rsm = m == 0 ? RS0 : RSW;
			// a streamed matrix's transposed A fragments (A[feature][neuron] = M^T rows of this wave's
			// tiles), loaded ahead so the latency hides behind the weight-gradient MFMAs
			h8 agT[MTW][W / 32];
			if (RA && streamed(m)) {
#pragma unroll
				for (int i = 0; i < MTW; ++i)
#pragma unroll
					for (int s = 0; s < W / 32; ++s) agT[i][s] = pagT[m >= 1 ? m - 1 : 0][i][s];
			} else if (PFB && streamed(m)) {
#pragma unroll
				for (int i = 0; i < MTW; ++i)
#pragma unroll
					for (int s = 0; s < W / 32; ++s) agT[i][s] = agTn[i][s];
			} else if (streamed(m)) {
				load_agT(m, agT);
			}
			if (PFB && m - 1 >= 1 && streamed(m - 1)) load_agT(m - 1, agTn);  // the next layer's, one layer ahead
			// dW_m += delta_{m+1} a_m^T (contraction over the tile's samples, 32 per MFMA)
#pragma unroll
			for (int i = 0; i < MTW; ++i)
#pragma unroll
				for (int kh = 0; kh < KH; ++kh) {
					const _Float16* amk = am + 32 * kh * rsm;
					if constexpr (SWZ0) {
						const h8 ad = trs(dsl + 32 * kh * RSW, wave * MTW + i);  // A[neuron][sample] (even/odd rows)
						if (m == 0) {
#pragma unroll
							for (int k = 0; k < KT0; ++k) dW0[i][k] = mfma16(ad, trsx(amk, k), dW0[i][k]);
						} else {
#pragma unroll
							for (int k = 0; k < L::MT; ++k) dWh[m > 0 ? m - 1 : 0][i][k] = mfma16(ad, trs(amk, k), dWh[m > 0 ? m - 1 : 0][i][k]);
						}
					} else {
						const h8 ad = trw(dsl + 32 * kh * RSW, wave * MTW + i);  // A[neuron][sample]
						if (m == 0) {
#pragma unroll
							for (int k = 0; k < KT0; ++k) dW0[i][k] = mfma16(ad, trx(amk, k), dW0[i][k]);
						} else {
#pragma unroll
							for (int k = 0; k < L::MT; ++k) dWh[m > 0 ? m - 1 : 0][i][k] = mfma16(ad, trw(amk, k), dWh[m > 0 ? m - 1 : 0][i][k]);
						}
					}
				}
			// delta_m = act'(a_m) * (M_m^T delta_{m+1})  (m == 0: dL/d(encoding), no transfer)
			const _Float16* Mt = streamed(m) ? nullptr : Wm(m);
			if (m > 0) {
#pragma unroll
				for (int i = 0; i < MTW; ++i) {
					const int t = wave * MTW + i;
					f4 v[NTAU];
#pragma unroll
					for (int tau = 0; tau < NTAU; ++tau) v[tau] = fz;
#pragma unroll
					for (int s = 0; s < W / 32; ++s) {
						const h8 af = streamed(m) ? agT[i][s] : trw(Mt + 32 * s * rsm, t);  // A[feature][neuron 32s+8q+e]
#pragma unroll
						for (int tau = 0; tau < NTAU; ++tau) v[tau] = mfma16(af, *(const h8*)(dsl + ixf(false, 16 * tau, 32 * s)), v[tau]);
					}
#pragma unroll
					for (int tau = 0; tau < NTAU; ++tau) dl[i][tau] = act_bwd<ACT>(*(const h4*)(am + ix4(16 * tau, 16 * t)), v[tau]);
				}
				if constexpr (!L::PP) __syncthreads();  // without the spare slot delta_m overwrites a_m, read above
				_Float16* dst = dslot(m);
#pragma unroll
				for (int i = 0; i < MTW; ++i)
#pragma unroll
					for (int tau = 0; tau < NTAU; ++tau) *(h4*)(dst + ix4(16 * tau, 16 * (wave * MTW + i))) = dl[i][tau];
				__syncthreads();
			} else if (a.dldenc) {
				for (int t = wave; t < KT0; t += WAVES) {
					f4 v[NTAU];
#pragma unroll
					for (int tau = 0; tau < NTAU; ++tau) v[tau] = fz;
#pragma unroll
					for (int s = 0; s < W / 32; ++s) {
						const h8 af = trx(Mt + 32 * s * RS0, t);
#pragma unroll
						for (int tau = 0; tau < NTAU; ++tau) v[tau] = mfma16(af, *(const h8*)(dsl + ixf(false, 16 * tau, 32 * s)), v[tau]);
					}
#pragma unroll
					for (int tau = 0; tau < NTAU; ++tau) {
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
			if (row < WR) {
#pragma unroll
				for (int k = 0; k < KT0; ++k) dst[row * IN + 16 * k + c] = dW0[i][k][r];
#pragma unroll
				for (int j = 0; j < NH - 1; ++j)
#pragma unroll
					for (int k = 0; k < L::MT; ++k)
						if (16 * k + c < WR) dst[WR * IN + j * WR * WR + row * WR + 16 * k + c] = dWh[j][i][k][r];
			}
		}
	}
#pragma unroll
	for (int i = 0; i < NTW; ++i)
#pragma unroll
		for (int r = 0; r < 4; ++r)
			if (16 * (wave * NTW + i) + c < WR) dst[WR * IN + (NH - 1) * WR * WR + (OP ? 4 * r + q : 4 * q + r) * WR + 16 * (wave * NTW + i) + c] = dWo[i][r];
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

// ---------------------------------------------------------------------------------------------
// inference
// ---------------------------------------------------------------------------------------------
// inference geometry (plain functions: also used in the kernel's launch bounds)
constexpr int tile_infer_nthr(int WR) { return 64 * (tile_kw(WR) / 32); }  // waves: two row tiles each
constexpr int tile_infer_T(int WR) { return tile_kw(WR) >= 128 ? 32 : 64; }  // samples per tile
// hidden matrices whose A fragments stay in registers: 176 VGPRs for A (W0: 8 per 32 inputs, Wout: 4
// per 32 neurons, hidden: 8 per 32 neurons)
constexpr int tile_infer_nrh(int WR, int IN, int NH) {
	return tile_imax(0, tile_imin(NH - 1, (176 - 8 * ((IN + 31) / 32) - 4 * (tile_kw(WR) / 32)) / (8 * (tile_kw(WR) / 32))));
}
constexpr int tile_infer_bytes(int WR, int IN, int NH) {
	return 2 * ((NH - 1 - tile_infer_nrh(WR, IN, NH)) * tile_kw(WR) * (tile_kw(WR) + 8) + tile_infer_T(WR) * ((IN + 31) / 32 * 32 + 8) +
	            2 * tile_infer_T(WR) * (tile_kw(WR) + 8));
}
constexpr int tile_infer_weu(int WR, int IN, int NH) {
	return tile_imax(1, tile_imax(1, tile_imin(8 / (tile_kw(WR) / 32), tile_lds_limit() / tile_infer_bytes(WR, IN, NH))) * (tile_kw(WR) / 32) / 4);
}

template <int WR, int IN, int NH>
struct TileInferLayout {
	static constexpr int W = tile_kw(WR);
	static constexpr int KP0 = (IN + 31) / 32 * 32, RS0 = KP0 + 8, RSW = W + 8;
	static constexpr int MT = W / 16, MTW = 2, WAVES = MT / MTW;  // W128 4 waves, W64 2, W32 (and W16) 1
	static constexpr int NTHR = 64 * WAVES;
	static constexpr int KS0 = KP0 / 32, KSW = W / 32;
	// A fragments kept in registers (VGPRs per wave): W0 and Wout always, hidden matrices 1..NRH while
	// the budget lasts (all of them for every instantiated shape); the rest are staged in LDS
	static constexpr int NRH = tile_infer_nrh(WR, IN, NH);
	static constexpr int NLH = NH - 1 - NRH;
	static constexpr int T = tile_infer_T(WR), NST = T / 16;  // samples per tile / 16-sample MFMA columns
	static constexpr int oWl = 0;                     // LDS hidden matrices NRH+1.. [NLH][W][RSW]
	static constexpr int oX = oWl + NLH * W * RSW;    // input tile [T][RS0]
	static constexpr int oP = oX + T * RS0;           // activation tiles [2][T][RSW]
	static constexpr int HALVES = oP + 2 * T * RSW;
	static constexpr int BYTES = HALVES * 2;
	static constexpr int WG_PER_CU = tile_imax(1, tile_imin(8 / WAVES, tile_lds_limit() / BYTES));
	static constexpr int WAVES_PER_EU = tile_imax(1, WG_PER_CU * WAVES / 4);
	static_assert(BYTES <= tile_lds_limit(), "tile inference exceeds the LDS");
	static_assert(BYTES == tile_infer_bytes(WR, IN, NH) && NTHR == tile_infer_nthr(WR) && WAVES_PER_EU == tile_infer_weu(WR, IN, NH),
	              "launch-bound helpers");
	static_assert(oX % 8 == 0 && oP % 8 == 0, "16-byte alignment");
};

struct TileInferArgs {
	uint32_t B;
	int out_act;
	const _Float16* params;  // [W0 | hidden | Wout] fp16 (unpadded width WR)
	const _Float16* enc;     // encoded input fp16 [B][IN]
	_Float16* out;           // network output fp16 [B][16]
};

template <int WR, int IN, int NH, Act ACT>
__global__ __launch_bounds__(tile_infer_nthr(WR), tile_infer_weu(WR, IN, NH)) void k_mlp_tile_infer(const TileInferArgs a) {
	using L = TileInferLayout<WR, IN, NH>;
	constexpr int W = L::W, MTW = L::MTW, WAVES = L::WAVES, NTHR = L::NTHR, T = L::T, NST = L::NST;
	constexpr int RS0 = L::RS0, RSW = L::RSW, KS0 = L::KS0, KSW = L::KSW, NRH = L::NRH;
	extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
	const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	const int c = lane & 15, q = lane >> 4;
	const f4 fz = {0.0f, 0.0f, 0.0f, 0.0f};
	_Float16* X = smem + L::oX;
	_Float16* P0 = smem + L::oP;
	_Float16* P1 = smem + L::oP + T * RSW;

	// ---- weight-stationary A fragments (rows 16 (wave MTW + i) + c, columns 32 s + 8 q ..+7) ----
	const _Float16* p = a.params;
	h8 aw0[MTW][KS0];
	h8 awh[NRH > 0 ? NRH : 1][MTW][KSW];
	h8 awo[KSW];
#pragma unroll
	for (int i = 0; i < MTW; ++i) {
		const int row = 16 * (wave * MTW + i) + c;
#pragma unroll
		for (int s = 0; s < KS0; ++s) {
			const int col = 32 * s + 8 * q;
			aw0[i][s] = (row < WR && col < IN) ? *(const h8*)(p + (size_t)row * IN + col) : zero8();
		}
#pragma unroll
		for (int j = 0; j < NRH; ++j)
#pragma unroll
			for (int s = 0; s < KSW; ++s) {
				const int col = 32 * s + 8 * q;
				awh[j][i][s] = (row < WR && col < WR) ? *(const h8*)(p + (size_t)WR * IN + ((size_t)j * WR + row) * WR + col) : zero8();
			}
	}
	const _Float16* pwo = p + (size_t)WR * IN + (size_t)(NH - 1) * WR * WR;
#pragma unroll
	for (int s = 0; s < KSW; ++s) awo[s] = 32 * s + 8 * q < WR ? *(const h8*)(pwo + (size_t)c * WR + 32 * s + 8 * q) : zero8();
	// hidden matrices beyond the register budget -> LDS
	for (int idx = tid; idx < L::NLH * W * (W / 8); idx += NTHR) {
		const int r = idx / (W / 8), c8 = idx % (W / 8);
		const int j = r / W + NRH, rr = r % W;
		*(h8*)(smem + L::oWl + r * RSW + 8 * c8) = (rr < WR && 8 * c8 < WR) ? *(const h8*)(p + (size_t)WR * IN + ((size_t)j * WR + rr) * WR + 8 * c8) : zero8();
	}
	// zero the padded input columns once (the input loads never write them)
	if (L::KP0 > IN)
		for (int idx = tid; idx < T * (L::KP0 - IN); idx += NTHR) X[(idx / (L::KP0 - IN)) * RS0 + IN + idx % (L::KP0 - IN)] = (_Float16)0.0f;

	constexpr int XV = T * IN / 8, XPT = (XV + NTHR - 1) / NTHR;
	const uint32_t n_tiles = (a.B + T - 1) / T;
	uint32_t tile = blockIdx.x;
	h8 xr[XPT];
	auto load_x = [&](uint32_t t) {
#pragma unroll
		for (int j = 0; j < XPT; ++j) {
			const int idx = tid + NTHR * j;
			const uint32_t row = t * T + idx / (IN / 8);
			if (idx < XV) xr[j] = row < a.B ? *(const h8*)(a.enc + (size_t)row * IN + 8 * (idx % (IN / 8))) : zero8();
		}
	};
	if (tile < n_tiles) load_x(tile);

	for (; tile < n_tiles; tile += gridDim.x) {
		const uint32_t base = tile * T;
#pragma unroll
		for (int j = 0; j < XPT; ++j) {
			const int idx = tid + NTHR * j;
			if (idx < XV) *(h8*)(X + (idx / (IN / 8)) * RS0 + 8 * (idx % (IN / 8))) = xr[j];
		}
		if (tile + gridDim.x < n_tiles) load_x(tile + gridDim.x);
		__syncthreads();

#pragma unroll
		for (int m = 0; m < NH; ++m) {
			const _Float16* in = m == 0 ? X : ((m - 1) & 1 ? P1 : P0);
			_Float16* outp = (m & 1) ? P1 : P0;
			const int rsi = m == 0 ? RS0 : RSW;
			const int KS = m == 0 ? KS0 : KSW;
			f4 acc[MTW][NST];
#pragma unroll
			for (int i = 0; i < MTW; ++i)
#pragma unroll
				for (int tau = 0; tau < NST; ++tau) acc[i][tau] = fz;
#pragma unroll
			for (int s = 0; s < KS; ++s) {
				h8 b[NST];
#pragma unroll
				for (int tau = 0; tau < NST; ++tau) b[tau] = *(const h8*)(in + (16 * tau + c) * rsi + 32 * s + 8 * q);
#pragma unroll
				for (int i = 0; i < MTW; ++i) {
					h8 af;
					if (m == 0) af = aw0[i][s];
					else if (m - 1 < NRH) af = awh[m - 1 < NRH ? m - 1 : 0][i][s];
					else af = *(const h8*)(smem + L::oWl + (m - 1 - NRH) * W * RSW + (16 * (wave * MTW + i) + c) * RSW + 32 * s + 8 * q);
#pragma unroll
					for (int tau = 0; tau < NST; ++tau) acc[i][tau] = mfma16(af, b[tau], acc[i][tau]);
				}
			}
#pragma unroll
			for (int i = 0; i < MTW; ++i)
#pragma unroll
				for (int tau = 0; tau < NST; ++tau)
					*(h4*)(outp + (16 * tau + c) * RSW + 16 * (wave * MTW + i) + 4 * q) = tile_act<ACT>(acc[i][tau]);
			__syncthreads();
		}

		// ---- output layer: 16 rows, one 16-sample tile per wave at a time ----
		const _Float16* aN = ((NH - 1) & 1) ? P1 : P0;
#pragma unroll
		for (int tau = wave; tau < NST; tau += WAVES) {
			f4 y = fz;
#pragma unroll
			for (int s = 0; s < KSW; ++s) y = mfma16(awo[s], *(const h8*)(aN + (16 * tau + c) * RSW + 32 * s + 8 * q), y);
			const uint32_t i = base + 16 * tau + c;
			if (i < a.B) *(h4*)(a.out + (size_t)i * 16 + 4 * q) = out_act_fwd(a.out_act, y);
		}
	}
}

// ---------------------------------------------------------------------------------------------
// per-width dispatch (mlp_tile_w*.hip)
// ---------------------------------------------------------------------------------------------
#define TCNN_TILE_SHAPES_OF(X, w) \
	X(w, 16, 1) X(w, 16, 2) X(w, 16, 3) X(w, 16, 4) X(w, 16, 5) \
	X(w, 32, 1) X(w, 32, 2) X(w, 32, 3) X(w, 32, 4) X(w, 32, 5) \
	X(w, 64, 1) X(w, 64, 2) X(w, 64, 3) X(w, 64, 4) X(w, 64, 5) \
	X(w, 128, 1) X(w, 128, 2) X(w, 128, 3) X(w, 128, 4) X(w, 128, 5)

struct TileShapeInfo {
	uint32_t lds_bytes, n_streamed, wg_per_cu, waves;  // training (the variant tile_ra_selected picks)
	uint32_t infer_lds_bytes, infer_wg_per_cu, infer_tile;
	uint32_t reg_a;                                    // 1: the register-resident training variant
	uint32_t ts64;                                     // 1: 64-sample tiles (batches that are a multiple of 64)
};

// whether the training launch of a shape with tile_ra_ok takes the register-resident variant (its
// default policy, TCNN_TILE_REG_A=0/1 overrides; read once per process)
bool tile_ra_selected(uint32_t W, uint32_t IN, uint32_t NH);
// whether shapes with tile_ts64_ok run 64-sample tiles (default; TCNN_TILE_SAMPLES=32 selects 32)
bool tile_ts64_selected();

// per-width entry points (one translation unit per width); false if (IN, NH) is not instantiated
bool tile_shape_w16(uint32_t IN, uint32_t NH, TileShapeInfo* info);
bool tile_shape_w32(uint32_t IN, uint32_t NH, TileShapeInfo* info);
bool tile_shape_w64(uint32_t IN, uint32_t NH, TileShapeInfo* info);
bool tile_shape_w128(uint32_t IN, uint32_t NH, TileShapeInfo* info);
// the in-kernel grid encode instantiation (mlp_tile_w128.hip): <128, 32, 4>, ReLU, 64-sample tiles
bool tile_train_w128_genc(hipStream_t st, HashType h, uint32_t blocks, const TileTrainArgs& a);
bool tile_train_w16(hipStream_t st, uint32_t IN, uint32_t NH, int act, uint32_t blocks, const TileTrainArgs& a);
bool tile_train_w32(hipStream_t st, uint32_t IN, uint32_t NH, int act, uint32_t blocks, const TileTrainArgs& a);
bool tile_train_w64(hipStream_t st, uint32_t IN, uint32_t NH, int act, uint32_t blocks, const TileTrainArgs& a);
bool tile_train_w128(hipStream_t st, uint32_t IN, uint32_t NH, int act, uint32_t blocks, const TileTrainArgs& a);
bool tile_infer_w16(hipStream_t st, uint32_t IN, uint32_t NH, int act, uint32_t blocks, const TileInferArgs& a);
bool tile_infer_w32(hipStream_t st, uint32_t IN, uint32_t NH, int act, uint32_t blocks, const TileInferArgs& a);
bool tile_infer_w64(hipStream_t st, uint32_t IN, uint32_t NH, int act, uint32_t blocks, const TileInferArgs& a);
bool tile_infer_w128(hipStream_t st, uint32_t IN, uint32_t NH, int act, uint32_t blocks, const TileInferArgs& a);

template <int WR, int IN, int NH>
inline void tile_info_fill(TileShapeInfo* info) {
	using L = TileLayout<WR, IN, NH>;
	using LI = TileInferLayout<WR, IN, NH>;
	*info = TileShapeInfo{(uint32_t)L::BYTES, (uint32_t)L::NS, (uint32_t)L::WG_PER_CU, (uint32_t)L::WAVES,
	                      (uint32_t)LI::BYTES, (uint32_t)LI::WG_PER_CU, (uint32_t)LI::T, 0u, 0u};
	if constexpr (tile_ra_ok(tile_kw(WR), IN, NH)) {
		if (tile_ra_selected(WR, IN, NH)) {
			using LR = TileLayout<WR, IN, NH, true>;
			info->lds_bytes = LR::BYTES, info->n_streamed = LR::NS, info->wg_per_cu = LR::WG_PER_CU, info->waves = LR::WAVES;
			info->reg_a = 1u;
			if constexpr (tile_ts64_ok(tile_kw(WR), IN, NH, true)) {
				if (tile_ts64_selected()) {
					using LR6 = TileLayout<WR, IN, NH, true, 64>;
					info->lds_bytes = tile_imax(LR::BYTES, LR6::BYTES), info->wg_per_cu = tile_imin(LR::WG_PER_CU, LR6::WG_PER_CU);
					info->ts64 = 1u;
				}
			}
			return;
		}
	}
	if constexpr (tile_ts64_ok(tile_kw(WR), IN, NH, false)) {
		if (tile_ts64_selected()) {
			// the 64-sample variant's layout; a batch that is not a multiple of 64 runs the 32-sample kernel,
			// which streams no more matrices (the transposed copy is sized for the larger count)
			using L6 = TileLayout<WR, IN, NH, false, 64>;
			info->lds_bytes = tile_imax(L::BYTES, L6::BYTES), info->n_streamed = L6::NS, info->wg_per_cu = tile_imin(L::WG_PER_CU, L6::WG_PER_CU);
			info->ts64 = 1u;
		}
	}
}

// the definitions of one width's entry points (used once per mlp_tile_w*.hip)
#define TCNN_TILE_WIDTH_TU(w)                                                                                                    \
	template <int IN, int NH, Act A, bool RA, int TS = 32>                                                                       \
	static void tile_train_launch_v_##w(hipStream_t st, uint32_t blocks, const TileTrainArgs& a) {                               \
		using L = TileLayout<w, IN, NH, RA, TS>;                                                                                 \
		static uint64_t done = 0;                                                                                                \
		set_dyn_lds((const void*)k_mlp_tile_train<w, IN, NH, A, RA, TS>, L::BYTES, done);                                        \
		hipLaunchKernelGGL((k_mlp_tile_train<w, IN, NH, A, RA, TS>), dim3(blocks), dim3(L::NTHR), L::BYTES, st, a);             \
	}                                                                                                                            \
	template <int IN, int NH, Act A>                                                                                             \
	static void tile_train_launch_##w(hipStream_t st, uint32_t blocks, const TileTrainArgs& a) {                                 \
		if constexpr (tile_ra_ok(tile_kw(w), IN, NH)) {                                                                          \
			if (tile_ra_selected(w, IN, NH)) {                                                                                   \
				if constexpr (tile_ts64_ok(tile_kw(w), IN, NH, true)) {                                                          \
					if (tile_ts64_selected() && a.B % 64 == 0) {                                                                 \
						tile_train_launch_v_##w<IN, NH, A, true, 64>(st, blocks, a);                                             \
						return;                                                                                                  \
					}                                                                                                            \
				}                                                                                                                \
				tile_train_launch_v_##w<IN, NH, A, true>(st, blocks, a);                                                         \
				return;                                                                                                          \
			}                                                                                                                    \
		}                                                                                                                        \
		if constexpr (tile_ts64_ok(tile_kw(w), IN, NH, false)) {                                                                 \
			if (tile_ts64_selected() && a.B % 64 == 0) {                                                                         \
				tile_train_launch_v_##w<IN, NH, A, false, 64>(st, blocks, a);                                                    \
				return;                                                                                                          \
			}                                                                                                                    \
		}                                                                                                                        \
		tile_train_launch_v_##w<IN, NH, A, false>(st, blocks, a);                                                                \
	}                                                                                                                            \
	template <int IN, int NH, Act A>                                                                                             \
	static void tile_infer_launch_##w(hipStream_t st, uint32_t blocks, const TileInferArgs& a) {                                 \
		using L = TileInferLayout<w, IN, NH>;                                                                                    \
		static uint64_t done = 0;                                                                                                \
		set_dyn_lds((const void*)k_mlp_tile_infer<w, IN, NH, A>, L::BYTES, done);                                                \
		hipLaunchKernelGGL((k_mlp_tile_infer<w, IN, NH, A>), dim3(blocks), dim3(L::NTHR), L::BYTES, st, a);                     \
	}                                                                                                                            \
	bool tile_shape_w##w(uint32_t IN, uint32_t NH, TileShapeInfo* info) {                                                        \
		TCNN_TILE_SHAPES_OF(TCNN_TILE_INFO_X, w)                                                                                 \
		return false;                                                                                                            \
	}                                                                                                                            \
	bool tile_train_w##w(hipStream_t st, uint32_t IN, uint32_t NH, int act, uint32_t blocks, const TileTrainArgs& a) {           \
		TCNN_TILE_SHAPES_OF(TCNN_TILE_TRAIN_X, w)                                                                                \
		return false;                                                                                                            \
	}                                                                                                                            \
	bool tile_infer_w##w(hipStream_t st, uint32_t IN, uint32_t NH, int act, uint32_t blocks, const TileInferArgs& a) {           \
		TCNN_TILE_SHAPES_OF(TCNN_TILE_INFER_X, w)                                                                                \
		return false;                                                                                                            \
	}

#define TCNN_TILE_INFO_X(w, in, nh)                                                                                              \
	if (IN == in && NH == nh) {                                                                                                  \
		tile_info_fill<w, in, nh>(info);                                                                                         \
		return true;                                                                                                             \
	}
#define TCNN_TILE_TRAIN_X(w, in, nh)                                                                                             \
	if (IN == in && NH == nh) {                                                                                                  \
		if (act == ACT_RELU) tile_train_launch_##w<in, nh, Act::ReLU>(st, blocks, a);                                            \
		else tile_train_launch_##w<in, nh, Act::None>(st, blocks, a);                                                            \
		return true;                                                                                                             \
	}
#define TCNN_TILE_INFER_X(w, in, nh)                                                                                             \
	if (IN == in && NH == nh) {                                                                                                  \
		if (act == ACT_RELU) tile_infer_launch_##w<in, nh, Act::ReLU>(st, blocks, a);                                            \
		else tile_infer_launch_##w<in, nh, Act::None>(st, blocks, a);                                                            \
		return true;                                                                                                             \
	}

}  // namespace tcnn_amd
