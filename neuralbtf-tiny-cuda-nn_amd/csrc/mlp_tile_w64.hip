// mlp_tile_w64.hip -- the tile engine's W64 instantiations (training + inference, every (IN, NH) of
// TCNN_TILE_SHAPES_OF), one translation unit per width so they compile in parallel. See mlp_tile.h.
#include "mlp_tile.h"

namespace tcnn_amd {
TCNN_TILE_WIDTH_TU(64)
}  // namespace tcnn_amd
