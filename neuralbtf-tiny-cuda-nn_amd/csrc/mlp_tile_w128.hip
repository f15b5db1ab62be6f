// mlp_tile_w128.hip -- the tile engine's W128 instantiations (training + inference, every (IN, NH) of
// TCNN_TILE_SHAPES_OF), one translation unit per width so they compile in parallel. See mlp_tile.h.
#include "mlp_tile.h"

namespace tcnn_amd {
TCNN_TILE_WIDTH_TU(128)

// configs[3]'s kernel with the grid encoding gathered in-kernel (mlp_tile.h GENC)
template <HashType H>
static void tile_train_genc_launch(hipStream_t st, uint32_t blocks, const TileTrainArgs& a) {
	using L = TileLayout<128, 32, 4, false, 64>;
	constexpr int GENC = 1 + (int)H;
	constexpr int bytes = tile_genc_base_bytes(L::BYTES) + tile_genc_extra_bytes(32, L::WAVES);
	static_assert(bytes <= tile_lds_limit(), "GENC LDS");
	static uint64_t done = 0;
	set_dyn_lds((const void*)k_mlp_tile_train<128, 32, 4, Act::ReLU, false, 64, GENC>, bytes, done);
	hipLaunchKernelGGL((k_mlp_tile_train<128, 32, 4, Act::ReLU, false, 64, GENC>), dim3(blocks), dim3(L::NTHR), bytes, st, a);
}
bool tile_train_w128_genc(hipStream_t st, HashType h, uint32_t blocks, const TileTrainArgs& a) {
	switch (h) {
		case HashType::CoherentPrime: tile_train_genc_launch<HashType::CoherentPrime>(st, blocks, a); return true;
		case HashType::Prime: tile_train_genc_launch<HashType::Prime>(st, blocks, a); return true;
		default: return false;
	}
}
}  // namespace tcnn_amd
