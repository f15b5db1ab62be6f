// mlp_tile_w16.hip -- the tile engine's W16 instantiations (training + inference, every (IN, NH) of
// TCNN_TILE_SHAPES_OF), one translation unit per width so they compile in parallel. See mlp_tile.h.
#include "mlp_tile.h"

namespace tcnn_amd {
TCNN_TILE_WIDTH_TU(16)
}  // namespace tcnn_amd
