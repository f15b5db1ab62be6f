// mlp_tile_w32.hip -- the tile engine's W32 instantiations (training + inference, every (IN, NH) of
// TCNN_TILE_SHAPES_OF), one translation unit per width so they compile in parallel. See mlp_tile.h.
#include "mlp_tile.h"

namespace tcnn_amd {
TCNN_TILE_WIDTH_TU(32)
}  // namespace tcnn_amd
