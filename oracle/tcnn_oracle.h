/*
 * tcnn_oracle.h -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity oracle and the CPU baseline for the MI355X engine. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product path never
 * links or calls it. Every function cites the reference file:line it restates
 * (paths relative to the reference tree, mandyxmq/NeuralBTF-tiny-cuda-nn @ 2025-01-27).
 *
 * Parity pinning: the RNG, seed derivation and Xavier draws are pinned against the reference's own
 * dependencies/pcg32/pcg32.h + std::seed_seq compiled on this host (oracle/ref_known_answers.cpp,
 * built into oracle/_ref/ by oracle/Makefile) and against the known answers recorded in SURVEY.md
 * §8(c). The grid index/hash helpers are pinned by the SURVEY §8(c) known answers. The kernels
 * themselves (grid.h, fully_fused_mlp.cu, adam.h) cannot run here (CUDA only), so their
 * restatements are pinned only through those helpers and the committed golden fixtures.
 *
 * Numerics: "ideal" mode -- fp16 storage exactly where the reference stores fp16 (encoding output,
 * hidden activations, network output, loss gradient, backprop temporaries, parameters), fp32
 * accumulation everywhere else. The grid forward reproduces the reference's fp16 FMA chain
 * bit-exactly (grid.h:144-163, vec.h:370-376).
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- fp16 helpers ---- */
uint16_t orc_f2h(float f);             /* round-to-nearest-even, subnormals kept */
float orc_h2f(uint16_t h);
void orc_f2h_array(const float* in, uint16_t* out, size_t n);
void orc_h2f_array(const uint16_t* in, float* out, size_t n);
uint16_t orc_hfma(uint16_t a, uint16_t b, uint16_t c); /* fused a*b+c, one rounding (__hfma) */

/* ---- PCG32 (dependencies/pcg32/pcg32.h:40-200) ---- */
typedef struct { uint64_t state, inc; } orc_pcg32;
void orc_pcg32_seed(orc_pcg32* r, uint64_t initstate, uint64_t initseq);
uint32_t orc_pcg32_next_uint(orc_pcg32* r);
float orc_pcg32_next_float(orc_pcg32* r);
void orc_pcg32_advance(orc_pcg32* r, int64_t delta);
/* std::seed_seq::generate as specified by the C++ standard ([rand.util.seedseq]) -- used by
 * trainer.h:52-55 to derive the trainer rng seed. */
void orc_seed_seq(const uint32_t* seeds, size_t n_seeds, uint32_t* out, size_t n_out);
/* generate_random_uniform (random.h:39-70): strided write order of generate_random_kernel, then
 * rng.advance(n). */
void orc_generate_uniform(orc_pcg32* r, size_t n, float* out, float lo, float hi);
/* GPUMatrix::initialize_xavier_uniform (gpu_matrix.h:284-299) on a [rows x cols] matrix. */
void orc_xavier_uniform(orc_pcg32* r, uint32_t rows, uint32_t cols, float* out, float scale);

/* ---- multiresolution grid (encodings/grid.h, common_device.h:631-868) ---- */
enum { ORC_GRID_HASH = 0, ORC_GRID_DENSE = 1, ORC_GRID_TILED = 2 };
enum { ORC_HASH_PRIME = 0, ORC_HASH_COHERENT_PRIME = 1, ORC_HASH_REVERSED_PRIME = 2 };
enum { ORC_INTERP_NEAREST = 0, ORC_INTERP_LINEAR = 1, ORC_INTERP_SMOOTHSTEP = 2 };
#define ORC_MAX_LEVELS 128
typedef struct {
	uint32_t n_pos_dims, n_features_per_level, n_levels, log2_hashmap_size, base_resolution;
	float per_level_scale;
	uint32_t grid_type, hash_type, interpolation;
	/* derived by orc_grid_init */
	uint32_t offsets[ORC_MAX_LEVELS + 1]; /* in entries (grid.h:688-719) */
	float scales[ORC_MAX_LEVELS];         /* grid_scale (common_device.h:709-714) */
	uint32_t res[ORC_MAX_LEVELS];         /* grid_resolution (common_device.h:716-718) */
	uint32_t n_params;                    /* offsets[L] * F */
	/* options (grid_interface.h:101-123, grid.h:284-298); ignored unless opts != 0 */
	uint32_t opts;
	float max_level;                      /* fraction of the levels */
	const float* max_level_gpu;           /* [B] per point, overrides max_level */
	uint32_t stochastic;                  /* stochastic interpolation in the backward */
} orc_grid;
int orc_grid_init(orc_grid* g);
uint32_t orc_grid_index(const orc_grid* g, uint32_t level, const uint32_t* pos_grid);
uint32_t orc_coherent_prime_hash(uint32_t d, const uint32_t* pos_grid);
/* random_val(seed, idx) (common_device.h:333-337): pcg32{seed}.advance(idx).next_float() */
float orc_random_val(uint32_t seed, uint32_t idx);
/* kernel_grid (grid.h:48-212): pos CM [D][B] (pos[i*D+d]); table fp16 [n_params];
 * enc SoA: enc[(l*F+f)*B + i]. */
void orc_grid_fwd(const orc_grid* g, uint32_t B, const float* pos, const uint16_t* table, uint16_t* enc);
/* kernel_grid_backward (grid.h:214-320) in ideal precision: grad[p] += float(half(w))*float(dLdy);
 * dL_dy SoA fp16 [(l*F+f)*B + i]; grad fp32 [n_params] is accumulated into (caller zeroes). */
void orc_grid_bwd(const orc_grid* g, uint32_t B, const float* pos, const uint16_t* dL_dy, float* grad);
/* same loop: per grid parameter, the sum of |update| and the number of updates (accumulated into) */
void orc_grid_bwd_stats(const orc_grid* g, uint32_t B, const float* pos, const uint16_t* dL_dy, float* abssum, uint32_t* count);
/* dL/dx fp32 [B][D] through the grid (grid.h:171-211 dy_dx + 322-349 backward_input);
 * dL_dy SoA fp16 [(l*F+f)*B + i] (F <= 4, D <= 8) */
void orc_grid_bwd_input(const orc_grid* g, uint32_t B, const float* pos, const uint16_t* table, const uint16_t* dL_dy,
                        float* dL_dx);
/* backward_backward_input (grid.h:351-627 kernels, 902-1026 host): given dL/d(dL/dx) fp32 [B][D],
 *   grad      += dL/dgrid        (kernel_grid_backward_input_backward_grid, grid.h:351-455), fp32
 *   dL_ddLdy   = dL/d(dL/dy)     fp32 [B][L*F] (kernel_grid_backward_input_backward_dLdoutput, :602-627)
 *   dL_dx      = dL/dx           fp32 [B][D]   (kernel_grid_backward_input_backward_input, :457-600)
 * dL_dy SoA fp16 [(l*F+f)*B + i]; any output may be NULL (D <= 8, F <= 8). */
void orc_grid_bwd_bwd(const orc_grid* g, uint32_t B, const float* pos, const uint16_t* table, const float* dL_ddLdx,
                      const uint16_t* dL_dy, float* grad, float* dL_ddLdy, float* dL_dx);

/* ---- fully fused MLP (src/fully_fused_mlp.cu:47-557, 635-891) ----
 * params fp16: W0 [W x IN] RM, W_1..W_{NH-1} [W x W] RM, Wout [OUTP x W] RM (contiguous).
 * input fp16: SoA [IN][B] (in[k*B+i], the grid's RM layout) if input_soa else CM (in[i*IN+k]).
 * out fp16 CM [OUTP][B] (out[i*OUTP+o]); hidden fp16 NH x CM [W][B] (post-activation) or NULL.
 * activation: hidden activation in bits 0-7, output activation in bits 8-15, Activation enum order
 * (common.h:126-136: None, ReLU, LeakyReLU, Exponential, Sine, Sigmoid, Squareplus, Softplus, Tanh;
 * common_device.h:102-297). orc_mlp_bwd's dL_dout is AFTER the output-activation transfer
 * (orc_act_bwd_output). */
uint32_t orc_mlp_n_params(uint32_t W, uint32_t IN, uint32_t NH, uint32_t OUTP);
/* reference-mimic fp16 accumulation on (1) / off (0, default): see g_mimic in tcnn_oracle.c */
void orc_set_mimic(int on);
/* orc_mlp_bwd's wgrad = sum_i |delta_i a_i| (on) / sum_i delta_i a_i (off, default): tolerance sizing */
void orc_set_abs_wgrad(int on);
/* in-place output-activation transfer of dL/dout given the network output (bits 8-15 of act) */
void orc_act_bwd_output(uint32_t act, size_t n, const uint16_t* out16, uint16_t* g16);
void orc_mlp_fwd(uint32_t W, uint32_t IN, uint32_t NH, uint32_t OUTP, uint32_t activation,
                 const uint16_t* params, uint32_t B, const uint16_t* input, int input_soa,
                 uint16_t* out, uint16_t* hidden, int n_threads);
/* backward (fully_fused_mlp.cu:150-259, 735-836 + cutlass_matmul.h:351-515): wgrad fp32 (same
 * layout as params, overwritten), dL_dinput fp16 in the input layout (or NULL). */
void orc_mlp_bwd(uint32_t W, uint32_t IN, uint32_t NH, uint32_t OUTP, uint32_t activation,
                 const uint16_t* params, uint32_t B, const uint16_t* input, int input_soa,
                 const uint16_t* hidden, const uint16_t* dL_dout, float* wgrad,
                 uint16_t* dL_dinput, int n_threads);

/* ---- OneBlob (encodings/oneblob.h:46-164) and Identity (encodings/identity.h:45-85) ----
 * x fp32 CM [D][B] (x[i*D+d]); out fp16 AoS [B][stride]: out[i*stride + d*n_bins + b], padding
 * columns [D*n_bins, D*n_bins + n_pad) = 1. Forward reproduces the reference's subwarp shuffle,
 * including its 32-lane wrap for n_bins > 32 (see tcnn_oracle.c). */
void orc_oneblob_fwd(uint32_t B, uint32_t D, uint32_t n_bins, const float* x, uint16_t* out, uint32_t stride, uint32_t n_pad);
/* kernel_one_blob_backward: dL/dx fp32 [B][D] from dL/dy fp16 AoS [B][stride] */
void orc_oneblob_bwd(uint32_t B, uint32_t D, uint32_t n_bins, const float* x, const uint16_t* dy, uint32_t stride, float* dx);
void orc_identity_fwd(uint32_t B, uint32_t D, float scale, float offset, const float* x, uint16_t* out, uint32_t stride,
                      uint32_t n_pad);

/* ---- RelativeL2 loss (losses/relative_l2.h:40-76) ----
 * pred fp16 CM [stride][B]; target fp32 CM [dims][B]; values fp32 CM [stride][B] (may be NULL);
 * grads fp16 CM [stride][B]. Returns sum of values (in double). */
double orc_relative_l2(uint32_t B, uint32_t stride, uint32_t dims, float loss_scale,
                       const uint16_t* pred, const float* target, float* values, uint16_t* grads);
/* ---- L2 loss (losses/l2.h:40-76), same layouts ---- */
double orc_l2(uint32_t B, uint32_t stride, uint32_t dims, float loss_scale,
              const uint16_t* pred, const float* target, float* values, uint16_t* grads);

/* ---- Adam (optimizers/adam.h:47-188) ---- */
typedef struct {
	float learning_rate, beta1, beta2, epsilon, l2_reg;
	float relative_decay, absolute_decay, clipping_magnitude, non_matrix_learning_rate_factor;
	int adabound, optimize_matrix_params, optimize_non_matrix_params;
} orc_adam_cfg;
void orc_adam_default(orc_adam_cfg* c);
/* One optimizer step; current_step is the optimizer's step AFTER its increment (adam.h:151). */
void orc_adam_step(const orc_adam_cfg* c, uint32_t n, uint32_t n_matrix, float loss_scale,
                   uint32_t current_step, float* w32, uint16_t* w16, const uint16_t* grad16,
                   float* m1, float* m2, uint32_t* steps);

/* ---- Trainer::training_step for NetworkWithInputEncoding<Grid | OneBlob | Identity, FullyFusedMLP> ----
 * (trainer.h:97-190, network_with_input_encoding.h:70-113). Param layout [MLP | grid].
 * Returns the loss sum (trainer.h:205-207). Gradients are rounded to fp16 (the reference's
 * m_param_gradients is __half) before Adam. run_optimizer=0 leaves params untouched. */
typedef struct {
	orc_grid grid;
	uint32_t W, NH, OUTP, n_output_dims, activation;
	orc_adam_cfg adam;
	uint32_t n_params, n_mlp_params, adam_step;
	float* w32; uint16_t* w16; uint16_t* grad16; float* grad32; float* m1; float* m2; uint32_t* steps;
	/* encoding: 0 = grid (above), 1 = OneBlob, 2 = Identity; IN = padded encoding width (set by the
	 * caller for OneBlob / Identity: n_dims * n_bins or n_dims, rounded up to 16) */
	uint32_t enc_type, n_dims, n_bins, IN;
	float enc_scale, enc_offset;
	uint32_t loss_type; /* 0 = RelativeL2, 1 = L2 */
} orc_model;
int orc_model_init(orc_model* m, uint32_t seed); /* allocate + Trainer::initialize_params */
void orc_model_free(orc_model* m);
double orc_train_step(orc_model* m, uint32_t B, const float* pos, const float* target,
                      int run_optimizer, int n_threads);
/* NetworkWithInputEncoding::inference: output fp16 CM [OUTP][B] */
void orc_model_inference(orc_model* m, uint32_t B, const float* pos, uint16_t* out, int n_threads);

#ifdef __cplusplus
}
#endif
