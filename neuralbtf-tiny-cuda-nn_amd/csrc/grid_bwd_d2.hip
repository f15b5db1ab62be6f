// grid_bwd_d2.hip -- LDS-privatised grid backward instantiated for D = 2 (grid_bwd_lds.h)
#include "grid_bwd_lds.h"

namespace tcnn_amd {
template void grid_bwd_f<2>(hipStream_t, uint32_t, HashType, int, uint32_t, dim3, size_t, uint32_t, const float*, uint32_t,
                             const _Float16*, const GridSlice*, float*, uint32_t, const LevelInfo*, uint32_t, uint32_t, uint32_t,
                             const GridBwdLaunch&);
}  // namespace tcnn_amd
