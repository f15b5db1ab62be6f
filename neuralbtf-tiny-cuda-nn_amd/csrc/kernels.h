// kernels.h -- host-side launchers of the gfx950 kernels (defined in kernels.hip).
#pragma once

#include "common.h"

namespace tcnn_amd {

struct LevelInfo;

// Work plan of the LDS-privatised grid backward: one item per (level, entry range, feature range);
// the item's int32 accumulators (end-begin) x nf fit in grid_bwd_slot_budget() LDS slots.
struct GridSlice {
	uint32_t level;
	uint32_t begin;  // entry range within the level
	uint32_t end;
	uint32_t f0;     // feature range [f0, f0 + nf)
	uint32_t nf;
};

// Binned backward of the grid levels whose accumulators do not fit the LDS (grid_bin.hip): the
// level's entries are cut into slices of 2^slice_log2 entries; every (point, corner) update is
// counting-sorted by slice into per-chunk record runs, then one workgroup per slice ("bucket")
// accumulates its records in LDS and writes (or applies Adam to) the slice's gradient.
struct GridBinLevel {
	uint32_t level;
	uint32_t slice_log2;
	uint32_t n_slices;
	uint32_t bucket_base;  // first global bucket of the level
};

struct GridBinArgs {
	const GridBinLevel* lv;  // [n_slots]
	uint32_t n_slots, n_buckets;
	uint32_t n_chunks, pts_per_chunk;  // point chunks of the bin pass (pts_per_chunk = GRID_BIN_RECS >> D)
	uint32_t acc_lds_bytes;            // accumulator bytes of the largest slice
	uint2* recs;     // [n_slots][n_chunks][GRID_BIN_RECS] {(w16 << 16) | entry-in-slice, dL/dy bits or point index}
	uint2* dir;      // [n_buckets][n_chunks] {first record of the bucket's run in the chunk, count}
	float* dysum;    // [n_slots][n_chunks][F] sum of |dL/dy| (fixed-point range of the level)
};
constexpr uint32_t GRID_BIN_RECS = 4096;        // records per (level, chunk) run
constexpr uint32_t GRID_BIN_MAX_SLICES = 2048;  // slices per level
constexpr uint32_t GRID_ACC_LDS_BYTES = 64 * 1024;  // accumulator budget of one slice

// Runtime activation codes of the layer-wise engine (reference Activation, common.h:126-136).
enum : int {
	ACT_NONE = 0, ACT_RELU = 1, ACT_LEAKY_RELU = 2, ACT_EXPONENTIAL = 3, ACT_SINE = 4, ACT_SIGMOID = 5,
	ACT_SQUAREPLUS = 6, ACT_SOFTPLUS = 7, ACT_TANH = 8,
};

// Layout of the grid backward's per-chunk fp32 partial slabs: level-major like the parameters, but
// within a level whose work items hold nf < F features the slab is feature-group-major
// ([F/nf][size][nf]) so every item writes one contiguous range. slab index of grid parameter p,
// level l, entry e, feature f (f0 = f - f % nf):  pbase[l] + f0 * size[l] + e * nf[l] + (f - f0).
// Points per chunk up to which the LDS grid backward keeps a chunk's dL/dy in registers
// (GRID_BWD_THREADS x GRID_BWD_PR, grid_bwd_lds.h): the faster path, so large batches take more chunks.
constexpr uint32_t GRID_BWD_REG_POINTS = 1024u * 32u;

struct GridSlabMap {
	uint32_t n_levels, log2F;
	uint32_t pbase[MAX_LEVELS + 1];  // offset_l * F
	uint32_t size[MAX_LEVELS];
	uint32_t nf[MAX_LEVELS];
};

__device__ __forceinline__ uint32_t grid_slab_index(const GridSlabMap* __restrict__ m, uint32_t p) {
	uint32_t l = 0;
	while (l + 1 < m->n_levels && p >= m->pbase[l + 1]) ++l;
	const uint32_t r = p - m->pbase[l];
	const uint32_t e = r >> m->log2F, f = r & ((1u << m->log2F) - 1u);
	const uint32_t nf = m->nf[l];
	const uint32_t f0 = f & ~(nf - 1u);
	return m->pbase[l] + f0 * m->size[l] + e * nf + (f - f0);
}

struct AdamArgs {
	uint32_t n, n_matrix;
	float loss_scale, grad_scale;  // grad_scale multiplies the fp32 gradient before fp16 rounding (1/N for N-rank sums)
	float lr, beta1, beta2, eps, l2_reg, rel_decay, abs_decay, clip, nonmat_lr_factor;
	float lower_lr_bound, upper_lr_bound;
	int opt_matrix, opt_nonmatrix;
	float inv_loss_scale;  // 1 / loss_scale when that is exact (power of two), else 0
	// parameter range [begin, n) of this launch; when part != nullptr the gradient of parameter i is
	// the fixed-order sum of n_parts partial slabs part[j * part_stride + (i - begin)] (written back
	// to grad32[i]) instead of grad32[i] (reduction fused into the optimizer)
	uint32_t begin;
	const float* part;
	uint32_t n_parts, part_stride;
	// bias-correction factors sqrt(1 - beta2^t) / (1 - beta1^t) precomputed on the device by the
	// same adam_bias_factor for t = 1 .. factor_n (factor_table[t - 1]); other t are computed per
	// parameter. Parameters carry their own step counts (adam.h:110-113), so without the table every
	// grid entry paid two powf -- the Adam epilogue of the binned backward was VALU-bound on them.
	const float* factor_table;
	uint32_t factor_n;
	// grid slabs: parameter i reads slab element grid_slab_index(part_map, i - begin) (nullptr: i - begin)
	const GridSlabMap* part_map;
};

// Optimizer state buffers (full parameter vector [network | encoding]).
struct AdamBuffers {
	float* w32;
	_Float16* w16;
	float* g32;      // fp32 gradient sums (written by fused-reduction epilogues)
	_Float16* g16;   // fp16 gradients (reference m_param_gradients)
	float* m1;
	float* m2;
	uint32_t* steps;
};

// Work carried by the grid backward launch (single-GPU trainer step): n_mlp_groups extra
// workgroups, on CUs the grid items leave free, each reduce one column block of the fused kernel's
// network-gradient slabs, run Adam on those network parameters and write them into the next step's
// fused weight image; workgroup 0 also sums the loss partials.
// Where a reduction writes the torch binding's finalised parameter gradient (grad_finalize_store,
// common.h) instead of fp32 sums: out (nullable; fp16, or fp32 if out_f32) at the parameter's index.
struct GradFinalize {
	void* out = nullptr;
	float s = 1.0f;
	int out_f32 = 0;
};

struct GridBwdEpilogue {
	int enabled;
	int apply_adam;          // 0: only the reduction (network gradients -> buf.g32, loss), for the
	                         // multi-GPU path where the all-reduce sits between reduction and Adam
	AdamArgs adam_mlp;       // range [0, n_mlp)
	AdamBuffers buf;
	// network-gradient tail
	uint32_t n_mlp_groups;   // extra workgroups (0 = none)
	const float* wpart;      // fused kernel slabs [n_wparts][n_mlp]
	uint32_t n_wparts, n_mlp;
	const float* lpart;      // loss partials [n_wparts]
	float* d_loss;
	// fused weight image (mlp_fused.h FusedLayout): W0 rows of RSI halves at 0, hidden rows of RSW
	// at oWh, output rows of RSW at oWo
	_Float16* wimage;
	uint32_t W, IN, NH, RSI, RSW, oWh, oWo;
	GradFinalize fin;        // apply_adam == 0: network gradients finalised into fin.out instead of buf.g32
};

// Fused train step (grid encoding -> MLP fwd -> RelativeL2 -> MLP bwd -> dW partials, dL/denc).
// With dout16 != NULL the loss is skipped and dL/d(output) fp16 [B][16] is read instead (Module::backward).
// Returns false if no fused kernel exists for this shape.
bool fused_train_supported(uint32_t W, uint32_t IN, uint32_t NH, uint32_t D, uint32_t F, uint32_t OUTP, int act, HashType h);
// Workgroups the fused launch uses (= partial slabs it writes) for this shape and batch.
uint32_t fused_train_waves();  // waves per workgroup of k_fused_train_grid
uint32_t fused_train_n_blocks(uint32_t W, uint32_t IN, uint32_t NH, uint32_t D, uint32_t dims, bool ext_dout, uint32_t B);
void launch_fused_train(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, uint32_t D, HashType h, int act,
                        uint32_t B, uint32_t dims, float loss_scale, const void* params16, const void* table16,
                        const float* pos, const float* target, void* out16, void* dLdenc_pairs,
                        float* wgrad_partial, float* loss_partial, const LevelInfo* levels, bool hash_grid,
                        Interp interp, uint32_t n_blocks, const void* dout16, const void* wimage, uint32_t loss_l2 = 0, bool inrange_index = false,
                        const void* enc16 = nullptr,  // enc16: the encoding read from memory, SoA [IN][B] (no gathers)
                        float dout_scale = 1.0f);     // dout16 is used as fp16(dout16 * dout_scale)
// LDS weight image of the fused kernels, built once per parameter update.
size_t fused_weight_image_bytes(uint32_t W, uint32_t IN, uint32_t NH);
void launch_pack_weights(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, const void* params16, void* image);

// Forward-only MLP (inference): in fp16 SoA [IN][B] or AoS [B][IN] -> out fp16 [B][16].
bool mlp_infer_supported(uint32_t W, uint32_t IN, uint32_t NH, uint32_t OUTP, int act);
// grid encoding + MLP forward in one kernel (k_fused_fwd_grid); wimage null: the LDS image is built from
// params16 (16-byte aligned); enc16 (nullable) receives the SoA encoding
void launch_fused_fwd(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, uint32_t D, HashType h, int act, uint32_t B,
                      const void* wimage, const void* params16, const void* table16, const float* pos, const LevelInfo* levels, bool hash_grid,
                      Interp interp, bool inrange_index, void* enc16, void* out16);
void launch_mlp_infer(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, int act, bool soa, uint32_t B,
                      const void* wimage, const void* in16, void* out16);
// out[b*n_out + o] = (float)in[b*in_stride + o]  (reference trim_and_cast_from, object.cu:60-67)
void launch_trim_cast(hipStream_t st, uint32_t B, uint32_t in_stride, uint32_t n_out, const void* in16, float* out);

// Grid forward (standalone; reference kernel_grid layout): out SoA [(l*F+f)*B + i] when soa, else
// AoS [i*out_stride + l*F + f].
void launch_grid_fwd(hipStream_t st, uint32_t D, uint32_t F, HashType h, uint32_t B, uint32_t L,
                     const float* pos, uint32_t pos_stride, const void* table16, void* out16, bool soa,
                     uint32_t out_stride, const LevelInfo* levels, bool hash_grid, Interp interp, const GridOpts& opts = GridOpts{});

// Grid backward: dLdy layout 0 = level-major pairs ([l][i][F] halves), 1 = SoA ([(l*F+f)*B + i]),
// 2 = AoS ([i*dy_stride + l*F + f]).
uint32_t grid_bwd_slot_budget();
// host_slices / host_levels: the work plan's host copies, passed by value as kernel arguments when
// they fit (grid_bwd_lds.h GridBwdTables)
void launch_grid_bwd(hipStream_t st, uint32_t D, uint32_t F, HashType h, uint32_t B, const float* pos,
                     uint32_t pos_stride, const void* dLdy16, int dy_layout, uint32_t dy_stride, const GridSlice* slices,
                     uint32_t n_slices, uint32_t n_chunks, float* partial, uint32_t partial_stride,
                     const LevelInfo* levels, bool hash_grid, Interp interp, const GridBwdEpilogue* ep = nullptr,
                     const GridOpts& opts = GridOpts{}, const GridSlice* host_slices = nullptr, const LevelInfo* host_levels = nullptr,
                     uint32_t n_levels = 0);
// Binned backward, pass 1: counting-sort the updates of the binned levels by slice (GridBinArgs).
void launch_grid_bin(hipStream_t st, uint32_t D, uint32_t F, HashType h, uint32_t B, const float* pos, uint32_t pos_stride,
                     const void* dLdy16, int dy_layout, uint32_t dy_stride, const LevelInfo* levels, bool hash_grid, Interp interp,
                     const GridBinArgs& a, const GridOpts& opts = GridOpts{});
// Binned backward, pass 2: one workgroup per slice sums its records in LDS (int32 fixed point scaled
// by the level's sum of |dL/dy|) and writes the fp32 gradient of grid parameter p to grad32[p] (grid
// parameter order) or, with adam != nullptr, applies Adam to parameter param_base + p.
struct GridAccAdam {
	AdamArgs a;
	AdamBuffers buf;
	uint32_t param_base;
	int write_grad32;  // also store the fp32 sum into buf.g32
};
void launch_grid_acc(hipStream_t st, uint32_t D, uint32_t F, uint32_t B, const void* dLdy16, int dy_layout, uint32_t dy_stride,
                     const LevelInfo* levels, const GridBinArgs& a, float* grad32, const GridAccAdam* adam);

// dL/dx fp32 [B][dx_stride] through the grid (reference grid.h:171-211 + 322-349), dy_dx recomputed
// from the table; dLdy in the launch_grid_bwd layouts.
void launch_grid_bwd_input(hipStream_t st, uint32_t D, uint32_t F, HashType h, uint32_t B, uint32_t L, const float* pos,
                           uint32_t pos_stride, const void* table16, const void* dLdy16, int dy_layout, uint32_t dy_stride, float* dx,
                           uint32_t dx_stride, const LevelInfo* levels, bool hash_grid, Interp interp, const GridOpts& opts = GridOpts{});
// Second-order grid gradients (reference grid.h:351-627, 902-1026): from dL/d(dL/dx) fp32 [B][D]
// and dL/dy (AoS fp16 [B][dy_stride], nullable) -> grad32 += dL/dgrid (fp32 atomics, nullable),
// dL/d(dL/dy) AoS fp16 [B][ddy_stride] (nullable), dL/dx fp32 [B][D] (nullable).
void launch_grid_bwd_bwd(hipStream_t st, uint32_t D, uint32_t F, HashType h, uint32_t B, uint32_t L, const float* pos,
                         uint32_t pos_stride, const void* table16, const float* dL_ddLdx, const void* dLdy16, uint32_t dy_stride,
                         float* grad32, void* dLddLdy16, uint32_t ddy_stride, float* dx, const LevelInfo* levels, bool hash_grid,
                         Interp interp, const GridOpts& opts = GridOpts{});
// fused weight-image geometry (FusedLayout) for the epilogue
void fused_image_layout(uint32_t W, uint32_t IN, uint32_t NH, uint32_t* RSI, uint32_t* RSW, uint32_t* oWh, uint32_t* oWo);

// out[c] = sum_j in[j*N + c] in block_column_sums order (G = 16 column blocks of 1024 threads):
// the network-gradient reduction of the sequential path, identical to the grid-backward tail's
void launch_column_sums(hipStream_t st, const float* in, uint32_t n_parts, uint32_t N, float* out);
// workgroups of the grid backward's network-gradient tail = column blocks of launch_column_sums (the
// same G in both keeps the two reductions' summation order identical); TCNN_MLP_TAIL_GROUPS overrides
uint32_t mlp_tail_groups();
// out[p] = sum_j in[j*stride + grid_slab_index(map, p)] (the grid backward's slabs, fixed order)
void launch_grid_slab_reduce(hipStream_t st, const float* in, uint32_t n_parts, uint32_t stride, uint32_t n, float* out,
                             const GridSlabMap* map, GradFinalize fin = {});
// out[p] = sum_j in[j*stride + p] (p < n). tmp: caller-owned device scratch of
// reduce_partials_tmp_floats(n_parts, n) floats (per workspace, so concurrent modules / streams /
// devices never share it)
size_t reduce_partials_tmp_floats(uint32_t n_parts, uint32_t n);
void launch_reduce_partials(hipStream_t st, const float* in, uint32_t n_parts, uint32_t stride, uint32_t n,
                            float* out, float* tmp);

// ---- tile engine (mlp_tile.h): fused MLP for W in {16, 32, 64, 128}, IN in {16, 32, 64, 128},
// 1..5 hidden layers, hidden activation None / ReLU, any output activation; encoded input fp16 [B][IN] ----
uint32_t tile_train_lds_bytes(uint32_t W, uint32_t IN, uint32_t NH);
bool tile_train_supported(uint32_t W, uint32_t IN, uint32_t NH, uint32_t outp, int act);
uint32_t tile_train_blocks(uint32_t B, uint32_t W, uint32_t IN, uint32_t NH);
// hidden matrices whose weights do not fit the LDS beside the rest (e.g. W128/H5/IN128: 2) are read from
// L2; their transposed copy needs tile_train_wT_bytes of device memory (0: every matrix is staged)
uint32_t tile_train_n_streamed(uint32_t W, uint32_t IN, uint32_t NH);
uint32_t tile_train_wT_bytes(uint32_t W, uint32_t IN, uint32_t NH);
// dldenc (optional): dL/d(encoding) as level-major pairs [IN/2][B] (dldenc_pairs) or AoS fp16 [B][IN]
// wT: tile_train_wT_bytes of scratch (nullptr when 0), rewritten from params16 by this launch
// out_act: output activation (ACT_*) applied to the output, its transfer applied to dL/d(output)
// The grid encoding gathered inside the tile kernel (enc16 == nullptr; r06): 2-D positions, the fp16
// table, the level table, hash type / flag and the in-range-index flag of a 2-feature grid
struct TileGridEnc {
	const float* pos;
	const void* table16;
	const LevelInfo* levels;
	HashType hash;
	uint32_t hash_grid, inrange;
};
// whether the tile kernel gathers the grid encoding itself for this shape / batch (8-wave W128 kernel,
// IN 32 = 16 levels x 2 features, 64-sample tiles; opt-in with TCNN_TILE_GENC=1, measured slower)
bool tile_train_genc_ok(uint32_t W, uint32_t IN, uint32_t NH, int act, uint32_t B, HashType h);
void launch_mlp_tile_train(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, int act, int out_act, uint32_t B, uint32_t dims,
                           float loss_scale, uint32_t loss_l2, const void* params16, const void* enc16, const float* target,
                           const void* dout16, void* out16, void* dldenc, int dldenc_pairs, float* wgrad_partial, float* loss_partial,
                           void* wT, const TileGridEnc* genc = nullptr);
// forward only (the reference's INFERENCE instantiation): enc16 fp16 [B][IN] -> out16 fp16 [B][16]
bool tile_infer_supported(uint32_t W, uint32_t IN, uint32_t NH, uint32_t outp, int act);
uint32_t tile_infer_blocks(uint32_t B, uint32_t W, uint32_t IN, uint32_t NH);
void launch_mlp_tile_infer(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, int act, int out_act, uint32_t B, const void* params16,
                           const void* enc16, void* out16);

// generate_random_uniform<float> (random.h:57-70) from pcg32 {state, inc} (not advanced here)
void launch_generate_uniform(hipStream_t st, uint64_t n, uint64_t state, uint64_t inc, float* out, float lo, float hi);
void launch_generate_logistic(hipStream_t st, uint64_t n, uint64_t state, uint64_t inc, float* out, float mean, float stddev);
// pert16[i] = fp16(out16[i] + noise[i]) (the Trainer's output perturbation)
void launch_add_perturbation(hipStream_t st, uint32_t n, const void* out16, const float* noise, void* pert16);
void launch_adam(hipStream_t st, const AdamArgs& a, float* w32, void* w16, const float* grad32, void* grad16,
                 float* m1, float* m2, uint32_t* steps);

void launch_cast_f32_f16(hipStream_t st, const float* in, void* out, size_t n);
void launch_cast_f16_f32(hipStream_t st, const void* in, float* out, size_t n);
// loss-scale arithmetic of the torch binding (modules.py:128-137): out = fp16(in * s); x /= s (fp32);
// out = fp16(in / s), stored as fp16 or widened to fp32
void launch_scale_f16(hipStream_t st, const void* in, void* out, float s, size_t n);
void launch_div_f32(hipStream_t st, float* x, float s, size_t n);
void launch_div_f16(hipStream_t st, const void* in, void* out, float s, size_t n, bool out_f32);
void launch_grad_finalize(hipStream_t st, const float* g, void* out, float s, size_t n, bool out_f32);

// RelativeL2 (standalone, reference relative_l2.h:40-76): pred fp16 [B][stride] -> values, grads
void launch_relative_l2(hipStream_t st, uint32_t B, uint32_t stride, uint32_t dims, float loss_scale,
                        const void* pred16, const float* target, float* values, void* grads16);

void launch_sum(hipStream_t st, const float* in, uint32_t n, float* out);

// ---- layer-wise MFMA MLP (mlp_layers.hip); activations sample-major fp16 [B][width] ----
bool layered_width_supported(uint32_t w);
// y[B][N] = act(x[B][K] w^T), w row-major [N][K]
void launch_layer_fwd(hipStream_t st, uint32_t B, uint32_t N, uint32_t K, const void* w16, const void* x16, void* y16, int act);
// dx[B][K] = act'(h) * (dy[B][N] w); h == nullptr: no transfer
// pairs = true (no transfer only): dX written as level-major fp16 pairs [K/2][B] (grid F = 2 encodings)
void launch_layer_bwd(hipStream_t st, uint32_t B, uint32_t N, uint32_t K, const void* w16, const void* dy16, const void* h16,
                      void* dx16, int act, bool pairs = false);
// in-place output-activation transfer: g[i] = act'(y[i]) g[i] over n elements
void launch_act_bwd_inplace(hipStream_t st, uint32_t n, int act, const void* y16, void* g16);
// partial[chunk][N][K] = sum over the chunk's samples of dy[i][n] x[i][k]
uint32_t wgrad_n_chunks(uint32_t B);
void launch_wgrad(hipStream_t st, uint32_t B, uint32_t N, uint32_t K, const void* dy16, const void* x16, float* partial,
                  uint32_t n_chunks);
uint32_t relative_l2_n_blocks(uint32_t B, uint32_t stride);
void launch_relative_l2_partial(hipStream_t st, uint32_t B, uint32_t stride, uint32_t dims, float loss_scale, const void* pred16,
                                const float* target, void* grads16, float* loss_partial, uint32_t loss_l2 = 0,
                                const float* pdf = nullptr);
// out[i] += in[i] (Accumulate-mode gradients)
void launch_add_f32(hipStream_t st, const float* in, float* out, size_t n);

// ---- OneBlob / Identity encodings (encodings.hip); output AoS fp16 [B][out_stride], padding = 1 ----
void launch_oneblob_fwd(hipStream_t st, uint32_t B, uint32_t D, uint32_t n_bins, const float* x, uint32_t x_stride, void* out16,
                        uint32_t out_stride, uint32_t n_pad);
// dL/dx fp32 [B][x_stride] from dL/dy fp16 AoS (kernel_one_blob_backward, oneblob.h:116-147)
void launch_oneblob_bwd(hipStream_t st, uint32_t B, uint32_t D, uint32_t n_bins, const float* x, uint32_t x_stride,
                        const void* dy16, uint32_t dy_stride, float* dx, uint32_t dx_stride);
void launch_identity_fwd(hipStream_t st, uint32_t B, uint32_t D, float scale, float offset, const float* x, uint32_t x_stride,
                         void* out16, uint32_t out_stride, uint32_t n_pad);
void launch_identity_bwd(hipStream_t st, uint32_t B, uint32_t D, float scale, const void* dy16, uint32_t dy_stride, float* dx,
                         uint32_t dx_stride);

void launch_probe_hfma(hipStream_t st, const void* a, const void* b, const void* c, void* out, uint32_t n_pairs);
// Diagnostic: the config_hash fused (pipelined) kernel with s_memtime phase stamps (prof: [blocks*8][8] u64).
void launch_fused_train_profile(hipStream_t st, uint32_t B, uint32_t dims, const void* params16, const void* table16,
                                const float* pos, const float* target, void* dLdenc, float* wgrad_partial,
                                float* loss_partial, const LevelInfo* levels, uint32_t n_blocks, const void* wimage,
                                unsigned long long* prof);
// Debug probe: runs one MFMA 16x16x32 f16 and two ds_read_b64_tr_b16 with known data.
void launch_probe(hipStream_t st, float* mfma_out, int16_t* tr_out);

}  // namespace tcnn_amd
