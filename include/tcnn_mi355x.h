/*
 * tcnn_mi355x.h -- C-ABI drop-in boundary of the MI355X (gfx950) hash-grid + fully-fused-MLP engine.
 *
 * Plain pointers and sizes only (no torch / C++ types). All data pointers are DEVICE pointers owned
 * by the caller unless stated otherwise; `stream` is a hipStream_t (NULL = default stream).
 * Every entry point catches C++ exceptions at the boundary and reports failure through its return
 * value (0 = success, nonzero / NULL = failure); the message is available from tcnn_last_error()
 * (thread-local). This mirrors the reference's exception behaviour (pybind maps them to
 * RuntimeError, reference bindings/torch/tinycudann/bindings.cpp).
 *
 * Two layers are exposed, each replacing one reference interface:
 *   (1) tcnn_module_*  -- the runtime FFI tcnn::cpp::Module (reference include/tiny-cuda-nn/cpp_api.h:50-117,
 *                         src/cpp_api.cu:30-167) that the PyTorch extension / NeuralBTF caller binds.
 *   (2) tcnn_trainer_* -- create_from_config() + Trainer::training_step / loss / inference
 *                         (reference include/tiny-cuda-nn/config.h:46-63, trainer.h:47-361,
 *                         object.h:147-179) used by mlp_learning_an_image.
 *
 * Matrix conventions (reference common.h:157-167): input fp32 [n x n_input_dims] row-major
 * (= CM [n_input_dims x n]); outputs / params are fp16 when precision is Fp16; n must be a multiple
 * of tcnn_batch_size_granularity() (256).
 */
#ifndef TCNN_MI355X_H
#define TCNN_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TCNN_PRECISION_FP32 0 /* tcnn::cpp::Precision::Fp32 (cpp_api.h:75-78) */
#define TCNN_PRECISION_FP16 1 /* tcnn::cpp::Precision::Fp16 */

typedef struct tcnn_module tcnn_module;   /* tcnn::cpp::Module* (cpp_api.h:86-112) */
typedef struct tcnn_context tcnn_context; /* tcnn::cpp::Context (cpp_api.h:82-84) */
typedef struct tcnn_trainer tcnn_trainer; /* TrainableModel {loss, optimizer, network, trainer} (config.h:46-51) */

/* ---- library / device (cpp_api.h:61-80; src/cpp_api.cu:41-62) ---- */
const char* tcnn_last_error(void);
const char* tcnn_version(void);
uint32_t tcnn_batch_size_granularity(void);       /* cpp::batch_size_granularity() */
int tcnn_cuda_device(void);                       /* cpp::cuda_device() */
int tcnn_set_cuda_device(int device);             /* cpp::set_cuda_device() */
void tcnn_free_temporary_memory(void);            /* cpp::free_temporary_memory() */
int tcnn_has_networks(void);                      /* cpp::has_networks() */
float tcnn_default_loss_scale(int precision);     /* cpp::default_loss_scale() */
int tcnn_preferred_precision(void);               /* cpp::preferred_precision() */
/* cpp::set_log_callback(fn) (cpp_api.h:70, src/cpp_api.cu:61-63; common_host.h:46-66): severity is
 * the reference's LogSeverity order (0 Info, 1 Debug, 2 Warning, 3 Error, 4 Success); NULL removes
 * the callback. Called synchronously from whichever thread logs. */
typedef void (*tcnn_log_callback_t)(int severity, const char* message, void* user);
void tcnn_set_log_callback(tcnn_log_callback_t callback, void* user);

/* generate_random_uniform<float>(stream, rng, n, out, lower, upper) (random.h:57-70): n floats in the
 * reference's strided order (4 per thread, thread i jumps 4i) from the pcg32 stream {*rng_state,
 * *rng_inc} (dependencies/pcg32/pcg32.h); the state is advanced by n on return, as rng.advance(n). */
/* generate_random_logistic (random.h:77-80): logit(u) * stddev * 0.551328895 + mean over the uniform
 * stream of tcnn_generate_random_uniform; the state advances by n. */
int tcnn_generate_random_logistic(void* stream, uint64_t* rng_state, uint64_t* rng_inc, uint64_t n, float* out, float mean, float stddev);
int tcnn_generate_random_uniform(void* stream, uint64_t* rng_state, uint64_t* rng_inc, uint64_t n, float* out, float lower,
                                 float upper);

/* ---- runtime module FFI (cpp_api.h:86-117) ---- */
/* cpp::create_network_with_input_encoding(n_input_dims, n_output_dims, encoding, network) */
tcnn_module* tcnn_create_network_with_input_encoding(uint32_t n_input_dims, uint32_t n_output_dims,
                                                     const char* encoding_json, const char* network_json);
/* cpp::create_network(n_input_dims, n_output_dims, network) (= Identity encoding + network) */
tcnn_module* tcnn_create_network(uint32_t n_input_dims, uint32_t n_output_dims, const char* network_json);
/* cpp::create_encoding(n_input_dims, encoding, requested_precision) */
tcnn_module* tcnn_create_encoding(uint32_t n_input_dims, const char* encoding_json, int precision);
void tcnn_module_destroy(tcnn_module* m);

/* Module::inference(stream, n, input, output, params) (cpp_api.h:91) */
int tcnn_module_inference(tcnn_module* m, void* stream, uint32_t n, const float* input, void* output, const void* params);
/* Module::forward(stream, n, input, output, params, prepare_input_gradients) -> Context (cpp_api.h:92) */
tcnn_context* tcnn_module_forward(tcnn_module* m, void* stream, uint32_t n, const float* input, void* output,
                                  const void* params, int prepare_input_gradients);
/* Module::backward(stream, ctx, n, dL_dinput?, dL_doutput, dL_dparams?, input, output, params) (cpp_api.h:93);
 * dL_dparams == NULL -> GradientMode::Ignore, else Overwrite. dL_dinput may be NULL. */
int tcnn_module_backward(tcnn_module* m, void* stream, const tcnn_context* ctx, uint32_t n, float* dL_dinput,
                         const void* dL_doutput, void* dL_dparams, const float* input, const void* output,
                         const void* params);
/* The torch binding's backward with its loss-scale arithmetic folded in (reference
 * bindings/torch/tinycudann/modules.py:128-138): dL_doutput (fp16) is multiplied by loss_scale and
 * rounded to fp16, the module's backward runs on it, dL_dinput (fp32) is divided by loss_scale and
 * dL_dparams = fp16(fp16 gradient / loss_scale) -- stored as fp16, or widened to fp32 when
 * dparams_fp32 (the gradient of fp32 master parameters cast to fp16 for the module) -- the same
 * values the binding computes with three torch operations. */
int tcnn_module_backward_scaled(tcnn_module* m, void* stream, const tcnn_context* ctx, uint32_t n, float* dL_dinput,
                                const void* dL_doutput, void* dL_dparams, const float* input, const void* output,
                                const void* params, float loss_scale, int dparams_fp32);
/* Module::backward_backward_input(stream, ctx, n, dL_ddLdinput, input, dL_doutput?, dL_dparams?,
 * dL_ddLdoutput?, dL_dinput?, params) (cpp_api.h:94): second-order gradients from dL/d(dL/dinput)
 * fp32 [n][n_input_dims]. Implemented by grid encodings (grid.h:902-1026); every other module
 * fails like the reference's DifferentiableObject (object.h:278-288). Returns without work when
 * both dL_ddLdoutput and dL_dparams are NULL (grid.h:913-915). */
int tcnn_module_backward_backward_input(tcnn_module* m, void* stream, const tcnn_context* ctx, uint32_t n,
                                        const float* dL_ddLdinput, const float* input, const void* dL_doutput,
                                        void* dL_dparams, void* dL_ddLdoutput, float* dL_dinput, const void* params);
void tcnn_context_destroy(tcnn_context* ctx);

/* GridEncoding::set_max_level / max_level / set_max_level_gpu (grid_interface.h:101-123), on a grid
 * encoding module or the grid of a NetworkWithInputEncoding module: levels above
 * max_level * n_levels output 0 and get no gradient (grid.h:69-91, 236-244). max_level_per_point is
 * a device pointer to n floats (one per point of every later call), or NULL. Modules without a grid
 * fail (status != 0). With masking or stochastic interpolation in effect, networks run on the
 * layer-wise engine. */
int tcnn_module_set_max_level(tcnn_module* m, float max_level);
float tcnn_module_max_level(tcnn_module* m);
int tcnn_module_set_max_level_gpu(tcnn_module* m, const float* max_level_per_point);

uint32_t tcnn_module_n_input_dims(const tcnn_module* m);
uint32_t tcnn_module_n_output_dims(const tcnn_module* m); /* padded width (cpp_api.cu:130) */
uint64_t tcnn_module_n_params(const tcnn_module* m);
int tcnn_module_param_precision(const tcnn_module* m);
int tcnn_module_output_precision(const tcnn_module* m);
/* Module::initialize_params(seed, params_full_precision, scale): pcg32{seed} (cpp_api.cu:133-136);
 * params_fp32 is a DEVICE pointer to n_params floats. */
int tcnn_module_initialize_params(tcnn_module* m, uint64_t seed, float* params_fp32, float scale);
/* hyperparams() / name() as JSON / plain strings; valid until the next call on this module. */
const char* tcnn_module_hyperparams(tcnn_module* m);
const char* tcnn_module_name(tcnn_module* m);

/* ---- workspace arena (gpu_memory.h:426-754: GPUMemoryArena, allocate_workspace, free_gpu_memory_arena) ----
 * One arena per stream (per device for the null stream): a virtual address range the size of the
 * device memory with physical memory mapped at its end as it grows, so addresses stay valid across
 * growth. Allocations are 128-byte aligned; free returns the interval to the stream's arena. */
void* tcnn_workspace_allocate(void* stream, uint64_t n_bytes);
int tcnn_workspace_free(void* stream, void* ptr);
int tcnn_free_workspace_arena(void* stream);
/* mapped bytes of the stream's arena; virtual_memory = 1 when it grows by mapping (VMM), 0 fallback */
int tcnn_workspace_arena_info(void* stream, uint64_t* mapped_bytes, int* virtual_memory);

/* ---- trainer: create_from_config + Trainer<float, __half, __half> (config.h:53-63, trainer.h) ---- */
/* config_json holds {"loss", "optimizer", "encoding", "network"}; seed as Trainer(seed=1337). */
tcnn_trainer* tcnn_trainer_create(uint32_t n_input_dims, uint32_t n_output_dims, const char* config_json, uint32_t seed);
void tcnn_trainer_destroy(tcnn_trainer* t);
/* Trainer::training_step(stream, input [n x n_in] fp32, target [n x n_out] fp32, run_optimizer) (trainer.h:163-190). */
int tcnn_trainer_training_step(tcnn_trainer* t, void* stream, uint32_t n, const float* input, const float* target,
                               int run_optimizer);
/* Data-parallel split of training_step(run_optimizer = 0): part 0 = forward + loss + MLP backward
 * with the network gradients final in gradients_fp32()[0, n_network_params) and the loss sum; part 1
 * = the grid backward filling gradients_fp32()[n_network_params, n_params). Between the two the
 * caller may all-reduce the network gradients on another stream while part 1 runs. Results are
 * bit-identical to training_step(run_optimizer = 0). */
int tcnn_trainer_training_step_part(tcnn_trainer* t, void* stream, uint32_t n, const float* input, const float* target, int part);
/* Trainer::optimizer_step(stream, loss_scale) (trainer.h:155-157) */
int tcnn_trainer_optimizer_step(tcnn_trainer* t, void* stream);
/* Trainer::forward / backward (trainer.h:97-153): the halves of training_step with the reference's
 * options. forward: data_pdf fp32 [n x n_out] or NULL; external_dL_dy fp16 [n x padded_output_width]
 * (loss-scaled, i.e. already multiplied by tcnn_default_loss_scale) or NULL, in which case the loss
 * is evaluated on target; prepare_input_gradients keeps what a dL/dinput backward needs. The context
 * holds the output fp16 [n x padded_output_width] and dL/doutput. backward: gradients of the
 * context's dL/doutput into gradients_fp32 (accumulate = 0: Overwrite, 1: Accumulate,
 * GradientMode, common.h), optional dL/dinput fp32 [n x n_in]; then tcnn_trainer_optimizer_step. */
typedef struct tcnn_trainer_context tcnn_trainer_context;  /* Trainer::ForwardContext (trainer.h:89-95) */
tcnn_trainer_context* tcnn_trainer_forward(tcnn_trainer* t, void* stream, uint32_t n, const float* input, const float* target,
                                           const float* data_pdf, const void* external_dL_dy, int prepare_input_gradients);
/* Trainer::forward with output perturbation (trainer.h:114-123): perturbation fp32 [n x padded_output_width]
 * (the caller's noise, e.g. tcnn_generate_random_logistic with stddev = perturbation_sigma) is added to
 * the output and the loss and its dL/doutput are evaluated on the perturbed output; the context's
 * output stays the unperturbed one. */
tcnn_trainer_context* tcnn_trainer_forward_perturbed(tcnn_trainer* t, void* stream, uint32_t n, const float* input, const float* target,
                                                     const float* data_pdf, const float* perturbation, int prepare_input_gradients);
/* gradient_mode: GradientMode (common.h) -- 0 Overwrite, 1 Accumulate, 2 Ignore (dL/dinput only; the
 * parameter gradients are left as they are) */
int tcnn_trainer_backward(tcnn_trainer* t, void* stream, const tcnn_trainer_context* ctx, uint32_t n, const float* input,
                          float* dL_dinput, int gradient_mode);
/* Trainer::loss(stream, ctx) (trainer.h:205-211): synchronises stream; 0 for an external-dL/dy context */
float tcnn_trainer_context_loss(tcnn_trainer* t, void* stream, const tcnn_trainer_context* ctx);
const void* tcnn_trainer_context_output(const tcnn_trainer_context* ctx);
const void* tcnn_trainer_context_doutput(const tcnn_trainer_context* ctx);
void tcnn_trainer_context_destroy(tcnn_trainer_context* ctx);
uint32_t tcnn_trainer_padded_output_width(const tcnn_trainer* t);
/* Adam on parameters [begin, end) only, counting as one optimizer step (data-parallel sharded
 * optimizer: each rank updates its shard of the reduce-scattered gradient sums; the caller then
 * all-gathers the fp16 parameters). Not in the reference, which has no multi-GPU path. */
int tcnn_trainer_optimizer_step_range(tcnn_trainer* t, void* stream, uint64_t begin, uint64_t end);
/* Data-parallel exchange over peer-mapped device memory (xGMI / same-device IPC), no collective
 * library: every rank of a node exports a blob of tcnn_dp_peer_blob_bytes() bytes (IPC handles of its
 * gradient, parameter and optimizer-state buffers and of its step counters), the caller gathers the
 * N blobs in rank order (any host transport) and every rank attaches them; from then on each
 * training_step(run_optimizer = 1) sums the ranks' gradient sums for this rank's 1/N shard directly
 * from the peers' memory, runs Adam on that shard (gradient scale 1/N) and copies the other shards'
 * updated fp16 parameters -- one C-ABI call per step, no host synchronisation. The optimizer state
 * is sharded like the RCCL sharded schedule (tcnn_trainer_dp_gather_state completes it). Detach is
 * collective (every rank calls it); a trainer attached to peers must be detached by every rank before
 * it is destroyed. A rank that does not arrive within the timeout (tcnn_trainer_dp_peer_set_timeout;
 * default TCNN_PEER_TIMEOUT_S or 300 s) raises an error at the next call instead of hanging the GPU.
 * A timeout while waiting for the gradients leaves the parameters untouched; a timeout while waiting
 * for the other ranks' updated shards leaves this rank's own shard updated and the others not, so the
 * ranks' parameters then differ: after any timeout restore every rank from a snapshot. */
uint64_t tcnn_dp_peer_blob_bytes(void);
int tcnn_trainer_dp_peer_export(tcnn_trainer* t, int nranks, int rank, void* blob);
int tcnn_trainer_dp_peer_attach(tcnn_trainer* t, const void* blobs);
int tcnn_trainer_dp_peer_detach(tcnn_trainer* t);
/* seconds a peer wait polls before it gives up (also changes the current attachment's waits) */
int tcnn_trainer_dp_peer_set_timeout(tcnn_trainer* t, double seconds);
/* Drop this rank's export / attachment without the collective barrier -- only before any exchange
 * step ran, e.g. when another rank failed to attach (the caller then falls back to another exchange). */
int tcnn_trainer_dp_peer_abandon(tcnn_trainer* t);
/* ---- data-parallel exchange inside the engine (not in the reference, which has no multi-GPU path;
 * SURVEY.md §5, §8(e)) ----
 * One process per GPU. Rank 0 creates a unique id, the caller broadcasts its TCNN_DP_ID_BYTES bytes
 * (e.g. over torch.distributed), every rank creates its communicator (RCCL over xGMI, loaded on first
 * use) on its current device and attaches it to its trainer. From then on every
 * tcnn_trainer_training_step(run_optimizer = 1) is the whole data-parallel step in one call on
 * `stream` (hipGraph-capturable): this rank's forward / backward, the fp32 gradient sum across ranks
 * on the communicator's stream (the network part overlapped with the grid backward), then Adam with
 * gradient scale 1/N -- on every parameter (sharded = 0), or on this rank's 1/N shard of the
 * reduce-scattered sum followed by an all-gather of the fp16 parameters (sharded = 1; the fp32
 * masters and Adam state then stay current on the shard only: tcnn_trainer_dp_gather_state before
 * serialize(with_optimizer)). The communicator must outlive its attachment (attach NULL to detach). */
#define TCNN_DP_ID_BYTES 128
typedef struct tcnn_dp_comm tcnn_dp_comm;
int tcnn_dp_unique_id(void* id);
tcnn_dp_comm* tcnn_dp_comm_create(const void* id, int nranks, int rank);
void tcnn_dp_comm_destroy(tcnn_dp_comm* c);
int tcnn_trainer_set_dp(tcnn_trainer* t, tcnn_dp_comm* c, int sharded);
int tcnn_trainer_dp_gather_state(tcnn_trainer* t, void* stream);
/* Trainer::loss(stream, ctx) of the last training step (trainer.h:205-207); synchronises `stream`. */
float tcnn_trainer_loss(tcnn_trainer* t, void* stream);
/* Device pointer to the last step's loss sum (fp32 scalar), for graph-friendly readback. */
const float* tcnn_trainer_loss_device(tcnn_trainer* t);
/* network->inference(stream, input, output fp32 [n x n_out]) (object.h:147-176) */
int tcnn_trainer_inference(tcnn_trainer* t, void* stream, uint32_t n, const float* input, float* output);
uint64_t tcnn_trainer_n_params(const tcnn_trainer* t);
uint64_t tcnn_trainer_n_network_params(const tcnn_trainer* t); /* MLP part; grid params follow */
/* Parameter buffers (trainer.h:325-336): fp32 master, fp16 params, fp16 gradients; plus the fp32
 * gradient sum the kernels produce (what a data-parallel all-reduce exchanges). */
float* tcnn_trainer_params_fp32(tcnn_trainer* t);
void* tcnn_trainer_params(tcnn_trainer* t);
void* tcnn_trainer_param_gradients(tcnn_trainer* t);
float* tcnn_trainer_gradients_fp32(tcnn_trainer* t);
/* Adam state buffers (adam.h:128-148): first / second moments fp32 and per-parameter step counts
 * uint32, [n_params] each (device pointers owned by the trainer). */
int tcnn_trainer_optimizer_state(tcnn_trainer* t, float** first_moments, float** second_moments, uint32_t** steps);
/* Data-parallel support: Adam reads grad_fp32 * grad_scale (set 1/N after a sum all-reduce). */
int tcnn_trainer_set_gradient_scale(tcnn_trainer* t, float scale);
/* The loss scale training_step / forward / optimizer_step use -- the reference's loss_scale argument of
 * Trainer::forward and Trainer::optimizer_step (trainer.h:97-160); default default_loss_scale<__half>
 * = 128 (common.h:232). */
int tcnn_trainer_set_loss_scale(tcnn_trainer* t, float loss_scale);
/* hipGraph replay of the single-GPU training step (the reference Trainer's CUDA graph,
 * trainer.h:163-190 / cuda_graph.h:52-178): off by default. While on, training_step with
 * run_optimizer = 1 replays a captured graph as long as the batch size, the input / target pointers,
 * the hyper-parameters and scales are unchanged, and re-captures otherwise; results are bit-identical
 * to the eager step. The stream may be the legacy null stream (the graph runs on a private stream,
 * ordered after and before the caller's with events). */
int tcnn_trainer_set_graph(tcnn_trainer* t, int on);
int tcnn_trainer_graph_stats(const tcnn_trainer* t, uint64_t* captures, uint64_t* replays);
/* Re-upload params from a host fp32 array (Trainer::set_params_full_precision, trainer.h:231-244). */
int tcnn_trainer_set_params_full_precision(tcnn_trainer* t, const float* host_params, uint64_t n);
/* Adam step counter (AdamOptimizer::step(), adam.h:200-202). */
/* Snapshot in the reference's format: the msgpack bytes of Trainer::serialize(with_optimizer)
 * (trainer.h:275-315, adam.h:278-299). Call with buf == NULL to get the size. */
int tcnn_trainer_serialize(tcnn_trainer* t, int with_optimizer, void* buf, uint64_t capacity, uint64_t* size);
/* Trainer::deserialize: msgpack bytes (or the JSON text of the same object, binaries as {"bytes": [...]},
 * gpu_memory_json.h:52-71); params_type "__half" or "float", optional optimizer state. */
int tcnn_trainer_deserialize(tcnn_trainer* t, const void* buf, uint64_t size);
/* Trainer::serialize(with_optimizer) as json (trainer.h:275-290): the JSON text of the same object,
 * binaries in nlohmann's {"bytes": [...], "subtype": null} form, NUL-terminated; *size includes the NUL.
 * Call with buf = NULL for the size. tcnn_trainer_deserialize accepts the text back. */
int tcnn_trainer_serialize_json(tcnn_trainer* t, int with_optimizer, char* buf, uint64_t capacity, uint64_t* size);
uint32_t tcnn_trainer_optimizer_step_count(const tcnn_trainer* t);
/* Trainer::update_hyperparams(json) (trainer.h:213-216): {"optimizer": {...}} fields update Adam
 * (adam.h:235-283: learning_rate, betas, epsilon, l2_reg, ...). */
int tcnn_trainer_update_hyperparams(tcnn_trainer* t, const char* params_json);
/* {"optimizer": Adam hyperparams, "loss": {"otype"}} as JSON; valid until the next call on this thread. */
const char* tcnn_trainer_hyperparams(tcnn_trainer* t);
/* Trainer::initialize_params (trainer.h:68-87): re-seed pcg32{seed_seq{seed}[0]}, re-initialise every
 * parameter, zero the optimizer state and its step counter. */
int tcnn_trainer_initialize_params(tcnn_trainer* t, uint32_t seed);
/* Trainer::initialize_params from the caller's pcg32 {state, inc} (the reference's m_rng, trainer.h:67-85,
 * which keeps advancing across re-initialisations): draws the n_params initial values from it and
 * returns the advanced state (by n_params) in *state. */
int tcnn_trainer_initialize_params_rng(tcnn_trainer* t, uint64_t* state, uint64_t inc);
/* Engine diagnostics: name of the path the trainer runs ("fused" / "layered" / "unsupported"), for
 * training and for network->inference ("fused": the whole MLP in one launch). */
const char* tcnn_trainer_engine(const tcnn_trainer* t);
const char* tcnn_trainer_inference_engine(const tcnn_trainer* t);
/* The same for a network module (NetworkWithInputEncoding / create_network); "encoding" for encodings. */
const char* tcnn_module_engine(const tcnn_module* m);
const char* tcnn_module_inference_engine(const tcnn_module* m);
/* set_max_level on the trainer model's grid encoding (see tcnn_module_set_max_level) */
int tcnn_trainer_set_max_level(tcnn_trainer* t, float max_level);

/* ---- per-phase hipEvent timing of training steps (measurement hook, not in the reference) ----
 * Between begin and end training_step records events around its phases on its stream:
 * 0 fused grid-encode + MLP fwd/loss/bwd kernel (layered engine: the whole fwd/bwd), 1 grid backward,
 * 2 reductions + Adam on the critical path, 3 join with the side stream (overlapped step) / loss sum.
 * end() synchronises the device and writes the mean ms per phase over the complete steps. */
int tcnn_trainer_profile_begin(tcnn_trainer* t);
/* same, recording phase events only on every `every`-th step (each event record idles the GPU briefly) */
int tcnn_trainer_profile_begin_sampled(tcnn_trainer* t, uint32_t every);
int tcnn_trainer_profile_end(tcnn_trainer* t, double* ms_per_phase, uint32_t n_phases, uint32_t* n_steps);

#ifdef __cplusplus
}
#endif
#endif /* TCNN_MI355X_H */
