/* debug_api.h -- TEST-ONLY diagnostic entry points of libtcnn_mi355x.so (not part of the
 * product C-ABI, include/tcnn_mi355x.h): MFMA / transpose-read layout probe, the fused kernel's
 * per-phase cycle build, the packed-fp16 FMA probe. Used by tests/test_gpu_probe.py and tools/diag_*.py;
 * no product code path calls them and they may change without notice. */
#ifndef TCNN_DEBUG_API_H
#define TCNN_DEBUG_API_H
#include "../../include/tcnn_mi355x.h"
#ifdef __cplusplus
extern "C" {
#endif

/* layout probe for the MFMA / transpose-read operand maps */
int tcnn_debug_probe(void* stream, float* mfma_out /* device [64*4] */, int16_t* tr_out /* device [64*8] */);
/* Diagnostic build of the config_hash fused kernel with s_memtime stamps: per-phase wave-cycle sums
 * (0 grid encode, 1 hidden layers fwd, 2 output+loss, 3 bwd through hidden layers + their dW,
 * 4 first-layer dW, 5 dL/dx + store, 6 prologue, 7 epilogue reduction), summed over all waves, written to
 * host_cycles8[16] (slots 8.. used by newer builds). */
int tcnn_debug_fused_phase_cycles(tcnn_trainer* t, void* stream, uint32_t n, const float* input, const float* target,
                                  uint64_t* host_cycles8);
/* out[i] = fma(a[i], b[i], c[i]) with the packed-fp16 FMA the grid forward uses (n_pairs half2 values) */
int tcnn_debug_hfma(void* stream, const void* a, const void* b, const void* c, void* out, uint32_t n_pairs);

/* Measurement only: attach the peer exchange as rank 0 of `nranks` ranks whose buffers are all this
 * trainer's own, so one process runs the per-rank kernels of an N-rank peer step (Adam on a 1/N shard
 * over N mirrors, the gather of N - 1 shards, the polls) without peers or links. The parameters it
 * then trains are meaningless; detach with tcnn_trainer_dp_peer_abandon. */
int tcnn_debug_peer_loopback(tcnn_trainer* t, int nranks);

#ifdef __cplusplus
}
#endif
#endif /* TCNN_DEBUG_API_H */
