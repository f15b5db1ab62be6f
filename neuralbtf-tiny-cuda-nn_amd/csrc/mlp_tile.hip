// mlp_tile.hip -- host side of the tile engine (kernels in mlp_tile.h, instantiated per width in
// mlp_tile_w{16,32,64,128}.hip): shape queries, launch geometry and the launchers.
#include "mlp_tile.h"

#include <cstdlib>

namespace tcnn_amd {

// Register-resident training variant (mlp_tile.h, tile_ra_ok): the default for every eligible shape;
// TCNN_TILE_REG_A=0 selects the LDS-staged kernel instead (A/B switch).
bool tile_ra_selected(uint32_t W, uint32_t IN, uint32_t NH) {
	static const int env = [] {
		const char* e = std::getenv("TCNN_TILE_REG_A");
		return e ? (std::atoi(e) != 0 ? 1 : 0) : -1;
	}();
	if (!tile_ra_ok((int)tile_kw((int)W), (int)IN, (int)NH)) return false;
	return env != 0;
}

bool tile_ts64_selected() {
	static const bool on = [] {
		const char* e = std::getenv("TCNN_TILE_SAMPLES");
		return !(e && std::atoi(e) == 32);
	}();
	return on;
}

static bool tile_shape(uint32_t W, uint32_t IN, uint32_t NH, TileShapeInfo* info) {
	switch (W) {
		case 16: return tile_shape_w16(IN, NH, info);
		case 32: return tile_shape_w32(IN, NH, info);
		case 64: return tile_shape_w64(IN, NH, info);
		case 128: return tile_shape_w128(IN, NH, info);
		default: return false;
	}
}

uint32_t tile_train_lds_bytes(uint32_t W, uint32_t IN, uint32_t NH) {
	TileShapeInfo i{};
	return tile_shape(W, IN, NH, &i) ? i.lds_bytes : 0u;
}

uint32_t tile_train_n_streamed(uint32_t W, uint32_t IN, uint32_t NH) {
	TileShapeInfo i{};
	return tile_shape(W, IN, NH, &i) ? i.n_streamed : 0u;
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
	TileShapeInfo i{};
	return outp == 16 && (act == ACT_NONE || act == ACT_RELU) && tile_shape(W, IN, NH, &i) && i.lds_bytes <= 160 * 1024;
}

bool tile_infer_supported(uint32_t W, uint32_t IN, uint32_t NH, uint32_t outp, int act) {
	TileShapeInfo i{};
	return outp == 16 && (act == ACT_NONE || act == ACT_RELU) && tile_shape(W, IN, NH, &i) && i.infer_lds_bytes <= 160 * 1024;
}

static uint32_t cu_count() {
	int dev = 0, n = 0;
	TCNN_HIP_CHECK(hipGetDevice(&dev));
	TCNN_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
	return n > 0 ? (uint32_t)n : 256u;
}

// Persistent workgroups: WG_PER_CU per CU (two waves per SIMD where the LDS allows: the W64 shapes run
// 2 workgroups of 4 waves -- the second hides the first's barrier and LDS latency, configs[1] 8,240 ->
// 10,468 steps/s, the sample's default 7,072 -> 9,380; 3 measured mixed, profiles/r02_tile_wg_per_cu.txt),
// capped by the tiles. TCNN_TILE_WG_PER_CU overrides (A/B switch, capped by the LDS fit).
uint32_t tile_train_blocks(uint32_t B, uint32_t W, uint32_t IN, uint32_t NH) {
	TileShapeInfo i{};
	if (!tile_shape(W, IN, NH, &i)) return 1;
	uint32_t per_cu = i.wg_per_cu;
	static const int env = [] {  // read once per process
		const char* e = std::getenv("TCNN_TILE_WG_PER_CU");
		return e ? std::atoi(e) : 0;
	}();
	if (env > 0) per_cu = std::min(std::max(1u, (uint32_t)env), std::max(1u, (160u * 1024u) / i.lds_bytes));
	const uint32_t ts = i.ts64 && B % 64 == 0 ? 64u : 32u;
	return std::max(1u, std::min(cu_count() * per_cu, B / ts));
}

bool tile_train_genc_ok(uint32_t W, uint32_t IN, uint32_t NH, int act, uint32_t B, HashType h) {
	// opt-in (TCNN_TILE_GENC=1): measured 1.5 % slower than the separate AoS pass for configs[3] (tile kernel
	// 563 -> 667 us against the pass's 122 us: the combine at each tile's start sits between two workgroup
	// barriers, on the critical path of a barrier-bound kernel; profiles/r06_configs3_genc_ab.txt)
	static const bool on = [] {
		const char* e = std::getenv("TCNN_TILE_GENC");
		return e && std::atoi(e) != 0;
	}();
	return on && W == 128 && IN == 32 && NH == 4 && act == ACT_RELU && B % 64 == 0 && tile_ts64_selected() &&
	       !tile_ra_selected(W, IN, NH) && (h == HashType::CoherentPrime || h == HashType::Prime);
}

void launch_mlp_tile_train(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, int act, int out_act, uint32_t B, uint32_t dims,
                           float loss_scale, uint32_t loss_l2, const void* params16, const void* enc16, const float* target,
                           const void* dout16, void* out16, void* dldenc, int dldenc_pairs, float* wgrad_partial, float* loss_partial,
                           void* wT, const TileGridEnc* genc) {
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
	a.out_act = out_act;
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
	if (genc) {
		TCNN_CHECK(!enc16 && tile_train_genc_ok(W, IN, NH, act, B, genc->hash), "tile train: in-kernel grid encode not available for this shape");
		a.gpos = genc->pos;
		a.gtable = (const uint32_t*)genc->table16;
		a.glevels = genc->levels;
		a.ghash = genc->hash_grid;
		a.ginrange = genc->inrange;
		ok = tile_train_w128_genc(st, genc->hash, blocks, a);
		TCNN_CHECK(ok, "tile train: in-kernel grid encode not instantiated");
		TCNN_HIP_CHECK(hipGetLastError());
		return;
	}
	switch (W) {
		case 16: ok = tile_train_w16(st, IN, NH, act, blocks, a); break;
		case 32: ok = tile_train_w32(st, IN, NH, act, blocks, a); break;
		case 64: ok = tile_train_w64(st, IN, NH, act, blocks, a); break;
		case 128: ok = tile_train_w128(st, IN, NH, act, blocks, a); break;
	}
	TCNN_CHECK(ok, "tile train: shape not instantiated");
	TCNN_HIP_CHECK(hipGetLastError());
}

uint32_t tile_infer_blocks(uint32_t B, uint32_t W, uint32_t IN, uint32_t NH) {
	TileShapeInfo i{};
	if (!tile_shape(W, IN, NH, &i)) return 1;
	const uint32_t n_tiles = (B + i.infer_tile - 1) / i.infer_tile;
	return std::max(1u, std::min(cu_count() * i.infer_wg_per_cu, n_tiles));
}

void launch_mlp_tile_infer(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, int act, int out_act, uint32_t B, const void* params16,
                           const void* enc16, void* out16) {
	TCNN_CHECK(tile_infer_supported(W, IN, NH, 16, act), "tile inference: unsupported shape");
	if (B == 0) return;
	TileInferArgs a{};
	a.B = B;
	a.out_act = out_act;
	a.params = (const _Float16*)params16;
	a.enc = (const _Float16*)enc16;
	a.out = (_Float16*)out16;
	const uint32_t blocks = tile_infer_blocks(B, W, IN, NH);
	bool ok = false;
	switch (W) {
		case 16: ok = tile_infer_w16(st, IN, NH, act, blocks, a); break;
		case 32: ok = tile_infer_w32(st, IN, NH, act, blocks, a); break;
		case 64: ok = tile_infer_w64(st, IN, NH, act, blocks, a); break;
		case 128: ok = tile_infer_w128(st, IN, NH, act, blocks, a); break;
	}
	TCNN_CHECK(ok, "tile inference: shape not instantiated");
	TCNN_HIP_CHECK(hipGetLastError());
}

}  // namespace tcnn_amd
