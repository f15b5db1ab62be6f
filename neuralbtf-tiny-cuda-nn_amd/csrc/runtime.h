// runtime.h -- host-side objects of the engine: JSON config -> grid encoding / fused MLP /
// NetworkWithInputEncoding / Trainer, device buffers, workspace. The C-ABI (capi.cpp) and the
// C++ template API (include/tiny-cuda-nn/*.h) are thin layers over these classes.
#pragma once

#include <json.hpp>

#include <array>
#include <cstdlib>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "common.h"
#include "grid_device.h"
#include "kernels.h"

namespace tcnn_amd {

using json = nlohmann::json;

// ---- host PCG32 (same stream semantics as the reference's dependencies/pcg32/pcg32.h) ----
struct Pcg32 {
	uint64_t state = 0x853c49e6748fea9bULL, inc = 0xda3e39cb94b95bdbULL;
	Pcg32() = default;
	explicit Pcg32(uint64_t initstate, uint64_t initseq = 1u) { seed(initstate, initseq); }
	void seed(uint64_t initstate, uint64_t initseq = 1u);
	uint32_t next_uint();
	float next_float();
	void advance(int64_t delta);
};

// ---- grow-only device allocation ----
struct DevBuf {
	void* p = nullptr;
	size_t bytes = 0;
	DevBuf() = default;
	DevBuf(const DevBuf&) = delete;
	DevBuf& operator=(const DevBuf&) = delete;
	~DevBuf();
	void reserve(size_t n);  // contents are not preserved
	void release();
	template <typename T> T* as() const { return (T*)p; }
};

bool ieq(const std::string& a, const std::string& b);

// Scratch of one grid backward (grow-only).
struct GridBwdBufs {
	DevBuf partial, recs, dir, dysum;
	uint32_t n_chunks = 0;  // LDS items: point chunks = slabs in `partial`
	int plan = 0;           // the LDS work plan the slabs in `partial` follow (GridEncodingHost::plans)
};
// LDS work plan of the grid backward: items, their device copy, and whether the chunk slabs are in
// parameter order (no GridSlabMap needed to read them)
struct GridPlan {
	std::vector<GridSlice> slices;
	DevBuf d_slices;
	bool identity = true;
	GridPlan() = default;
	GridPlan& operator=(const GridPlan& o) {
		slices = o.slices;
		identity = o.identity;
		return *this;
	}
};
enum : int { PLAN_RANGE = 0, PLAN_FEATURE = 1 };

// ---- multiresolution grid (reference encodings/grid.h:652-1208) ----
// The engine's A/B and tuning switches (TCNN_* environment variables). Read once when an engine
// object is built -- never per step -- so an experiment sets them before creating its trainer or
// module. Process-wide debug switches (TCNN_DEBUG_POISON, TCNN_DEBUG_GRID_TIMES, TCNN_TILE_REG_A,
// TCNN_TILE_WG_PER_CU) are read once per process where they are used.
struct EngineSwitches {
	bool no_fused_grid = false;     // TCNN_NO_FUSED_GRID: grid models train on the tile engine
	bool no_tile_engine = false;    // TCNN_NO_TILE_ENGINE: FullyFusedMLP shapes train on the layer-wise engine
	bool no_inrange_index = false;  // TCNN_NO_INRANGE_INDEX: the generic grid index in every kernel
	bool split_encode = false;      // TCNN_SPLIT_ENCODE: the encoding as its own pass (experiment)
	bool no_forward_keep = false;   // TCNN_NO_FORWARD_KEEP: Module backward recomputes the forward
	bool split_forward = false;     // TCNN_SPLIT_FORWARD: grid forward + k_mlp_infer instead of k_fused_fwd_grid
	bool grid_bin_all = false;      // TCNN_GRID_BIN=all: bin every grid level that does not fit whole
	uint32_t grid_bwd_chunks = 0;   // TCNN_GRID_BWD_CHUNKS: grid backward point chunks (0: automatic)
	uint32_t grid_bwd_ranges = 0;   // TCNN_GRID_BWD_RANGES: at least this many entry ranges per hashed level (tuning)
	int grid_bwd_plan = -1;         // TCNN_GRID_BWD_PLAN=range|feature: force one work plan (A/B; -1: by batch)
	static EngineSwitches from_env();
};

struct GridEncodingHost {
	EngineSwitches sw = EngineSwitches::from_env();
	GridDesc desc{};
	uint32_t n_features = 0;     // L * F
	uint32_t n_to_pad = 0;       // alignment padding (reference set_padded_output_width)
	uint32_t n_params = 0;       // offset[L] * F
	bool stochastic = false;
	float max_level = 1000.0f;              // GridEncoding::set_max_level (grid_interface.h:101-107)
	const float* max_level_gpu = nullptr;   // set_max_level_gpu: [B] per point (grid_interface.h:109-123)
	std::vector<LevelInfo> levels;
	// backward plan: levels [0, first_binned) are LDS work items (`slices`, per-chunk slabs), levels
	// [first_binned, L) go through the binned backward (grid_bin.hip), one slot each
	GridPlan plans[2];  // PLAN_RANGE, PLAN_FEATURE (ctor); both have the same items when no level splits
	uint32_t first_binned = 0;
	bool inrange_index_ok = false;  // grid_index_inrange is exact for in-range positions (ctor)
	uint32_t n_lds_params = 0;  // offset[first_binned] * F
	std::vector<GridBinLevel> bin_levels;
	uint32_t n_buckets = 0, acc_lds_bytes = 0;
	DevBuf d_levels, d_slab_map, d_bin_levels;

	GridEncodingHost(uint32_t n_dims_to_encode, const json& enc);
	uint32_t padded_output_width() const { return n_features + n_to_pad; }
	void set_alignment(uint32_t a) { n_to_pad = (n_features + a - 1) / a * a - n_features; }
	bool hash_grid() const { return desc.grid_type == GridType::Hash; }
	// GridEncodingTemplated::initialize_params (grid.h:1059-1062) -> host fp32
	void initialize_params(Pcg32& rng, float* host_out, float scale = 1.0f) const;
	json hyperparams() const;
	const LevelInfo* dev_levels() const { return d_levels.as<LevelInfo>(); }
	GridOpts opts() const {
		GridOpts o;
		o.max_level = max_level;
		o.max_level_gpu = max_level_gpu;
		o.stochastic = stochastic ? 1u : 0u;
		o.n_features = n_features;
		const float t = (max_level * (float)n_features) / (float)desc.n_features_per_level + 1e-3f;
		o.active = (stochastic || max_level_gpu || (float)(desc.n_levels - 1) >= t) ? 1u : 0u;
		o.inrange_index = (inrange_index_ok && desc.interp == Interp::Linear && !sw.no_inrange_index) ? 1u : 0u;
		return o;
	}
	// the slabs' element order under a plan; nullptr when it is the parameter order (every LDS item holds
	// all F features of its entries: the readers then index the slabs directly, no dependent map load)
	const GridSlabMap* slab_map(int plan) const { return plans[plan].identity ? nullptr : d_slab_map.as<GridSlabMap>(); }
	// the plan of a launch: TCNN_GRID_BWD_PLAN=range|feature, else the range plan while the items x
	// chunks run in one round on the CUs (2^15 .. 2^18 points), the feature plan beyond (configs[3])
	int plan_for(uint32_t B, uint32_t reserved = 0) const {
		if (sw.grid_bwd_plan >= 0) return sw.grid_bwd_plan;
		const uint32_t n_items = (uint32_t)plans[PLAN_RANGE].slices.size();
		return (uint64_t)bwd_chunks(B, reserved) * n_items + reserved <= 256 ? PLAN_RANGE : PLAN_FEATURE;
	}
	// point chunks of the backward: items x chunks workgroups of 1024 threads (one per CU: 128 KiB
	// of LDS each) fit the CUs left after `reserved` other workgroups in ONE round, with one chunk of
	// slack (config_hash, 26 items + 16 tail workgroups: 7 / 8 / 9 / 10 chunks -> 68.8 / 65.8 /
	// 67.5 / 109 us, the last spilling into a second round); >= 4096 points each
	uint32_t bwd_chunks(uint32_t B, uint32_t reserved = 0) const {
		const std::vector<GridSlice>& slices = plans[PLAN_RANGE].slices;  // (both plans: the same count for F = 2)
		if (slices.empty()) return 1;
		const uint32_t n_cu = 256;
		const uint32_t fit = (n_cu > reserved ? n_cu - reserved : 1u) / (uint32_t)slices.size();
		uint32_t c = std::max(1u, fit > 2 ? fit - 1 : fit);
		// large batches: chunks small enough for the register-resident path, over several rounds
		// (configs[3], 2^20 points: 8 -> 32 chunks, grid backward 170 -> 99 us, step -4 %,
		// profiles/r04_grid_bwd_chunks.txt); config_hash at 2^18 keeps its 8
		c = std::max(c, (B + GRID_BWD_REG_POINTS - 1) / GRID_BWD_REG_POINTS);
		if (sw.grid_bwd_chunks) return std::max(1u, std::min(std::min(sw.grid_bwd_chunks, 32u), B / 1024));  // tuning override
		// >= 8192 points per chunk: below that the per-chunk slab (written here, read by Adam or the
		// slab reduction) costs more than the parallelism gains (2^15 points, one rank of N = 8:
		// 4 chunks 46.6 us per step vs 8 chunks 48.0, profiles/r05_chunk_sweep.txt)
		return std::max(1u, std::min(std::min(c, 32u), B / 8192));
	}
	// bin-pass geometry for B points (reserves the record / directory buffers in w)
	GridBinArgs bin_args(GridBwdBufs& w, uint32_t B) const;
	// The backward pieces. dy: dL/d(encoding) fp16 in launch_grid_bwd layout `layout` (stride for AoS).
	//   backward_items  LDS items -> per-chunk slabs in w.partial (+ the trainer's epilogue workgroups)
	//   backward_bin    bin pass of the binned levels
	//   backward_acc    accumulate pass: fp32 gradient of the binned levels into grad32 (grid
	//                   parameter order, whole grid vector) or Adam on them (adam != nullptr)
	//   reduce_items    fixed-order slab sums of the LDS levels into grad32[0, n_lds_params)
	// backward() = all four: the fp32 gradient of every grid parameter into grad32 [n_params].
	void backward_items(hipStream_t st, GridBwdBufs& w, uint32_t B, const float* pos, uint32_t pstride, const void* dy, int layout,
	                    uint32_t dy_stride, const GridBwdEpilogue* ep = nullptr, uint32_t reserved = 0) const;
	void backward_bin(hipStream_t st, GridBwdBufs& w, uint32_t B, const float* pos, uint32_t pstride, const void* dy, int layout,
	                  uint32_t dy_stride) const;
	void backward_acc(hipStream_t st, GridBwdBufs& w, uint32_t B, const void* dy, int layout, uint32_t dy_stride, float* grad32,
	                  const GridAccAdam* adam = nullptr) const;
	void reduce_items(hipStream_t st, GridBwdBufs& w, float* grad32, GradFinalize fin = {}) const;
	void backward(hipStream_t st, GridBwdBufs& w, uint32_t B, const float* pos, uint32_t pstride, const void* dy, int layout,
	              uint32_t dy_stride, float* grad32) const;
};

// ---- fully fused MLP shape (reference networks/fully_fused_mlp.h) ----
struct MlpHost {
	uint32_t width = 64, n_input = 32, n_hidden_layers = 2, n_output = 16, padded_output = 16;
	int activation = 1, output_activation = 0;
	std::string otype = "FullyFusedMLP";
	MlpHost() = default;
	MlpHost(uint32_t n_input_dims, uint32_t n_output_dims, const json& net);
	uint32_t n_params() const {
		return n_hidden_layers == 0 ? padded_output * n_input
		                            : width * n_input + (n_hidden_layers - 1) * width * width + padded_output * width;
	}
	void initialize_params(Pcg32& rng, float* host_out, float scale = 1.0f) const;  // Xavier (gpu_matrix.h:284-299)
	json hyperparams() const;
};

struct AdamHost {
	float learning_rate = 1e-3f, beta1 = 0.9f, beta2 = 0.999f, epsilon = 1e-8f, l2_reg = 1e-8f;
	float relative_decay = 0.0f, absolute_decay = 0.0f, clipping_magnitude = 0.0f, non_matrix_learning_rate_factor = 1.0f;
	bool adabound = false, optimize_matrix_params = true, optimize_non_matrix_params = true;
	void update(const json& p);
	json hyperparams() const;
};

// Encodings of the network input (reference encodings/*.h): the multiresolution grid (parametric,
// fused path), OneBlob (oneblob.h) and Identity (identity.h).
enum class EncKind { Grid, OneBlob, Identity };

struct EncodingHost {
	EncKind kind = EncKind::Grid;
	std::unique_ptr<GridEncodingHost> grid;
	uint32_t n_dims = 0;        // input dims encoded
	uint32_t n_bins = 16;       // OneBlob
	float scale = 1.0f, offset = 0.0f;  // Identity
	uint32_t n_to_pad = 0;      // OneBlob / Identity padding (grid: grid->n_to_pad)

	EncodingHost(uint32_t n_dims_to_encode, const json& enc);
	static bool known(const std::string& otype);
	uint32_t n_output_unpadded() const;
	uint32_t padded_output_width() const { return kind == EncKind::Grid ? grid->padded_output_width() : n_output_unpadded() + n_to_pad; }
	void set_alignment(uint32_t a);
	uint32_t n_params() const { return kind == EncKind::Grid ? grid->n_params : 0u; }
	void initialize_params(Pcg32& rng, float* host_out, float scale = 1.0f) const;
	json hyperparams() const;
	// encoded output AoS fp16 [B][padded_output_width()] (padding: grid 0, OneBlob / Identity 1)
	void forward_aos(hipStream_t st, uint32_t B, const float* x, const void* params16, void* out16) const;
	// dL/dx fp32 [B][n_dims] from dL/d(encoding) fp16 AoS; params16 = the encoding's parameters (grid)
	// dy16: AoS [B][padded width]; grid encodings also take dy_layout 0 (level-major pairs [L][B])
	void backward_input(hipStream_t st, uint32_t B, const float* x, const void* dy16, float* dx, const void* params16 = nullptr,
	                    int dy_layout = 2) const;
};

// Workspace for one fwd/bwd over a batch of B (sizes grow only).
struct StepWorkspace {
	DevBuf dLdenc, wgrad_partial, loss_partial, grad32_tmp, out16, enc16, wimage;
	GridBwdBufs gbw;
	DevBuf acts, delta0, delta1, dout16, red_tmp;  // layer-wise engine
	DevBuf tile_wT;  // tile engine: transposed copy of the streamed hidden matrices
	DevBuf loss_sum;  // the grid backward epilogue's loss sum where nobody reads it (fwd_bwd_fused)
	uint32_t n_fused_blocks = 0, n_loss_partials = 0;
	bool wimage_valid = false;  // fused weight image matches the current fp16 params (trainer fast path)
};

// NetworkWithInputEncoding<__half> (reference network_with_input_encoding.h:41-190) over two engines:
//   "fused"   grid encoding + W in {32, 64} FullyFusedMLP: one register-resident kernel
//             (mlp_fused.h) + the LDS-privatised grid backward;
//   "fused"   (tile) W in {16, 32, 64, 128} FullyFusedMLP with any encoding (mlp_tile.h), training
//             and inference;
//   "layered" everything else (CutlassMLP, other widths, output activations):
//             per-layer MFMA kernels (mlp_layers.hip) with fp16 activations in HBM.
struct NetworkHost {
	EngineSwitches sw = EngineSwitches::from_env();
	// the fused kernel reads an external dL/dy as fp16(dL/dy * ext_dout_scale): the torch binding's loss
	// scale folded into the load (set only around a Module backward, tcnn_module_backward_scaled)
	float ext_dout_scale = 1.0f;
	// set by the torch binding's backward (tcnn_module_backward_scaled): the fused engine writes the
	// finalised parameter gradient there from its reductions; grad_fin_done reports that it did
	GradFinalize grad_fin{};
	bool grad_fin_done = false;
	std::unique_ptr<EncodingHost> enc;
	GridEncodingHost* grid = nullptr;  // enc->grid when the encoding is a grid
	MlpHost mlp;
	uint32_t n_input_dims = 0, n_output_dims = 0;
	uint32_t loss_l2 = 0;  // training loss: 0 RelativeL2 (relative_l2.h), 1 L2 (l2.h)
	NetworkHost(uint32_t n_in, uint32_t n_out, const json& enc, const json& net);
	uint64_t n_params() const { return (uint64_t)mlp.n_params() + enc->n_params(); }
	bool fused_ok() const;   // register-resident kernel (mlp_fused.h): grid input, W <= 64
	bool tile_shape_ok() const;  // tile kernels (mlp_tile.h): FullyFusedMLP W in {16..128}, any encoding, IN <= 128, H <= 5
	bool tile_ok() const;        // the training engine is the tile kernel (tile_shape_ok and not fused_ok)
	bool tile_infer_ok() const;  // inference runs the tile inference kernel
	bool layered_ok() const;
	const char* engine() const { return (fused_ok() || tile_ok()) ? "fused" : layered_ok() ? "layered" : "unsupported"; }
	const char* inference_engine() const;  // "fused" (one MLP launch) or "layered"
	void initialize_params(Pcg32& rng, float* host_out, float scale = 1.0f) const;  // network first (nwie.h:124-130)

	// params16: [mlp | encoding] fp16. out16: fp16 [B][padded_output].
	// trust_image: ws.wimage_valid tracks params16 (the Trainer's own parameters, whose every writer
	// clears it), so a valid fused weight image is reused instead of re-packed
	void inference(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const void* params16, void* out16,
	               bool trust_image = false);
	// Forward that keeps what the backward needs (the reference's forward context, cpp_api.cu:84-109,
	// network_with_input_encoding.h:70-81): the encoding, in the layout of the engine the backward will
	// run (with_dinput: the caller wants dL/dinput) -- SoA [IN][B] for the register-resident grid kernel,
	// AoS [B][IN] for the tile kernel -- into keep (grown here). Returns the layout kept (KEEP_*); the
	// layer-wise engine keeps nothing (its backward recomputes the forward).
	enum : int { KEEP_NONE = 0, KEEP_FUSED_SOA = 1, KEEP_TILE_AOS = 2 };
	int backward_engine_keep(bool with_dinput) const;
	void fused_forward(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const void* params16, bool use_image, void* enc_soa,
	                   void* out16);
	int forward_keep(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const void* params16, void* out16, bool with_dinput,
	                 DevBuf& keep);
	// forward+backward; dout16 == nullptr -> RelativeL2 on target, else external dL/dout.
	// Writes fp32 gradient sums into grad32 ([mlp | encoding]) and the loss partials
	// (ws.loss_partial[0 .. ws.n_loss_partials)). dL_dinput (optional): fp32 [B][n_input_dims].
	// kept / kept_layout: a forward_keep encoding of this batch (used when the layout matches the engine).
	void fwd_bwd(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const float* target, uint32_t dims,
	             float loss_scale, const void* params16, const void* dout16, void* out16, float* grad32,
	             const std::function<void(int)>& mark = nullptr, float* dL_dinput = nullptr, const void* kept = nullptr,
	             int kept_layout = KEEP_NONE);
	json hyperparams() const;

	// pieces of the fused engine for the trainer's overlapped step
	void fused_kernel(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const float* target, uint32_t dims,
	                  float loss_scale, const void* params16, bool pack, const void* dout16 = nullptr, void* out16 = nullptr,
	                  const void* enc_soa = nullptr);
	void grid_backward(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, GridBwdEpilogue* ep = nullptr);
	void pack_weights(hipStream_t st, StepWorkspace& ws, const void* params16);

private:
	void fwd_bwd_fused(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const float* target, uint32_t dims,
	                   float loss_scale, const void* params16, const void* dout16, void* out16, float* grad32,
	                   const std::function<void(int)>& mark, const void* enc_soa);
	void fwd_bwd_tile(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const float* target, uint32_t dims,
	                  float loss_scale, const void* params16, const void* dout16, void* out16, float* grad32,
	                  const std::function<void(int)>& mark, float* dL_dinput, const void* enc_aos);
	void fwd_bwd_layered(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const float* target, uint32_t dims,
	                     float loss_scale, const void* params16, const void* dout16, void* out16, float* grad32,
	                     const std::function<void(int)>& mark, float* dL_dinput);
	// forward through the layers from ws.enc16; hidden activations kept in ws.acts when `keep`
	void forward_layers(hipStream_t st, StepWorkspace& ws, uint32_t B, const void* params16, void* out16, bool keep);
};

// Per-phase hipEvent timing of the training step (bench.py's live per-kernel roofline source).
// Phases on the trainer's stream: [0] fused grid+MLP kernel (fwd, loss, bwd, dW), [1] grid backward
// (two-launch step: with the reduction + Adam epilogue), [2] reductions, [3] loss sum / optimizer
// (sequential path only; phases a step does not have are skipped). Events are recorded
// only on every `every`-th step (each record is a barrier packet that idles the GPU for a few us).
struct PhaseTimer {
	static constexpr int N_PHASES = 4;
	bool enabled = false;
	uint32_t every = 1, counter = 0;
	bool sampling = false;  // this step records events
	std::vector<hipEvent_t> pool;
	std::vector<std::array<int, N_PHASES + 1>> marks;  // event indices per step (-1 = not recorded)
	size_t next = 0;
	hipEvent_t get();
	void reset() { next = 0; marks.clear(); }
	~PhaseTimer();
};

// One RCCL communicator of a data-parallel job (dp.cpp): rank `rank` of `nranks`, one process per
// GPU; collectives run on its own stream `cs`, joined to the trainer's stream with events.
struct DpComm {
	void* comm = nullptr;  // ncclComm_t
	int nranks = 1, rank = 0;
	hipStream_t cs = nullptr;
	hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
	DpComm(const void* unique_id, int nranks, int rank);
	~DpComm();
	DpComm(const DpComm&) = delete;
	DpComm& operator=(const DpComm&) = delete;
	void all_reduce_f32(float* buf, size_t n, hipStream_t st);
	// in place: rank r receives the sum of [r per, (r + 1) per) at buf + r per
	void reduce_scatter_f32(float* buf, size_t per, hipStream_t st);
	// in place: rank r's [r per, (r + 1) per) elements of elem_bytes (2 or 4) to every rank
	void all_gather(void* buf, size_t per_elems, int elem_bytes, hipStream_t st);
};
void dp_unique_id(void* id128);  // ncclGetUniqueId (one rank; the caller broadcasts it)

// Trainer::forward's context (reference trainer.h:89-95, 97-144): the network output, the loss-scaled
// dL/d(output) (from the loss, or the caller's external dL/dy), the loss partial sums and the encoding
// kept for the backward (NetworkHost::forward_keep).
struct TrainerFwdCtx {
	uint32_t B = 0;
	DevBuf keep;
	int layout = 0;
	DevBuf out16, dLdy16, lpart;
	DevBuf pert16;              // output + perturbation, what the loss saw (trainer.h:114-123)
	const void* ext = nullptr;  // external dL/dy (not owned)
	uint32_t n_lpart = 0;
	const void* dLdy() const { return ext ? ext : dLdy16.p; }
};

// Stream-ordered workspace arena (arena.cpp; reference gpu_memory.h:426-754)
void* workspace_allocate(hipStream_t st, size_t n_bytes);
void workspace_free(hipStream_t st, void* p);
void workspace_arena_free(hipStream_t st);
void workspace_arena_free_all();
uint64_t dp_peer_blob_bytes();  // bytes of one rank's peer-exchange blob (dp_peer.hip)
double peer_default_timeout_s();  // TCNN_PEER_TIMEOUT_S or 300 s
void workspace_arena_info(hipStream_t st, uint64_t* mapped_bytes, int* vmm);

struct TrainerHost {
	uint32_t n_input_dims, n_output_dims;
	PhaseTimer timer;
	json config;
	std::unique_ptr<NetworkHost> model;
	AdamHost adam;
	std::string loss_otype;
	uint64_t n_params = 0, n_mlp = 0;
	DevBuf w32, w16, g16, g32, m1, m2, steps, d_loss;
	// Adam bias-correction factors of steps 1 .. ftable_valid (AdamArgs::factor_table), for the betas
	// they were computed with; grown by doubling
	DevBuf d_ftable;
	std::vector<float> h_ftable;  // host staging of the table (computed on the host, see adam_args_table)
	uint32_t ftable_cap = 0, ftable_valid = 0;
	float ftable_b1 = 0.0f, ftable_b2 = 0.0f;
	// makes the table cover steps 1 .. upto (computing what is missing, 1024 steps ahead) and
	// returns args with factor_table / factor_n set
	// (capacity for at least `reserve` entries)
	AdamArgs adam_args_table(hipStream_t st, uint32_t upto, uint32_t reserve = 0);
	StepWorkspace ws;
	uint32_t adam_step = 0;
	float grad_scale = 1.0f;       // what Adam multiplies the fp32 gradient sum by
	float grad_scale_user = 1.0f;  // the caller's factor (tcnn_trainer_set_gradient_scale); x 1/N under set_dp
	float loss_scale = 128.0f;  // default_loss_scale<__half> (common.h:232)
	uint32_t last_B = 0;
	// two-launch single-GPU step: reductions + Adam fused into the grid backward's epilogue
	bool overlapped_ok() const { return model->fused_ok(); }
	// grad_out (run_optimizer = false only): where the fp32 gradient sums go (default g32)
	void training_step_overlapped(hipStream_t st, uint32_t B, const float* input, const float* target, bool run_optimizer,
	                              float* grad_out = nullptr, bool skip_reduce = false);
	AdamArgs adam_args() const;

	TrainerHost(uint32_t n_in, uint32_t n_out, const json& cfg, uint32_t seed);
	void initialize_params(uint32_t seed);
	void initialize_params_rng(Pcg32& rng);  // from the caller's generator (advanced by n_params draws)
	void training_step(hipStream_t st, uint32_t B, const float* input, const float* target, bool run_optimizer);
	void step_eager(hipStream_t st, uint32_t B, const float* input, const float* target);  // with the optimizer
	void training_step_sequential(hipStream_t st, uint32_t B, const float* input, const float* target, bool run_optimizer);
	void training_step_part(hipStream_t st, uint32_t B, const float* input, const float* target, int part);
	void optimizer_step(hipStream_t st);
	// Trainer::forward / backward (trainer.h:97-153): the two halves of training_step with the
	// reference's options -- data_pdf (fp32 [B][n_output_dims]), external dL/dy (fp16 [B][padded
	// output], loss-scaled like the loss's own), dL/dinput (fp32 [B][n_input_dims]) and Accumulate
	// gradients (added to gradients_fp32() instead of overwriting it). Gradients land in the buffer
	// optimizer_step() reads.
	// perturbation (nullable): fp32 [B][padded output] noise added to the output before the loss
	std::unique_ptr<TrainerFwdCtx> forward(hipStream_t st, uint32_t B, const float* input, const float* target, const float* pdf,
	                                       const void* ext_dLdy16, bool prep_dinput, const float* perturbation = nullptr);
	// gradient_mode: 0 Overwrite, 1 Accumulate, 2 Ignore (GradientMode, common.h)
	void backward(hipStream_t st, const TrainerFwdCtx& c, uint32_t B, const float* input, float* dL_dinput, int gradient_mode);
	float ctx_loss(hipStream_t st, const TrainerFwdCtx& c);
	DevBuf g32_acc;  // Accumulate mode: this backward's gradients before they are added
	// data-parallel exchange inside the step (dp.cpp): with a communicator attached every
	// training_step(run_optimizer = true) sums the gradients across the ranks (all-reduce, or
	// reduce-scatter + Adam on this rank's shard + all-gather of the fp16 parameters when sharded)
	DpComm* dp = nullptr;
	bool dp_sharded = false, dp_state_partial = false;
	uint64_t dp_per = 0;  // parameters per shard (sharded: buffers padded to nranks * dp_per)
	void set_dp(DpComm* c, bool sharded);
	void training_step_dp(hipStream_t st, uint32_t B, const float* input, const float* target);
	void dp_gather_state(hipStream_t st);
	// data-parallel exchange over peer-mapped device memory, no collective library (dp_peer.hip):
	// export IPC handles of this rank's buffers, attach every rank's, then each training_step exchanges
	// through the peers' memory (sharded Adam, fp16 parameter gather)
	struct PeerDp;
	std::shared_ptr<PeerDp> peer;
	bool peer_attached = false;
	void dp_peer_export(int nranks, int rank, void* blob);
	void dp_peer_attach(const void* blobs);
	void dp_peer_detach();
	void dp_peer_loopback(int nranks);  // measurement only: an N-rank attachment whose peers are all this rank
	void dp_peer_abandon();  // local, no barrier: only before any exchange step (a failed attach on some rank)
	double peer_timeout_s = peer_default_timeout_s();
	void dp_peer_set_timeout(double seconds);
	void peer_check() const;  // throws if a wait of an earlier step failed
	int peer_nranks = 1;  // ranks of the attached peer exchange
	// ranks whose gradients Adam's input sums (RCCL communicator or peer exchange): grad_scale = user / N
	int dp_nranks() const { return dp ? dp->nranks : (peer_attached ? peer_nranks : 1); }
	void dp_peer_gather_state(hipStream_t st);
	void training_step_peer(hipStream_t st, uint32_t B, const float* input, const float* target);
	void peer_wait(hipStream_t st, int c, int slot, int signal_bump = -1, long long timeout_ticks = -1);  // -1: the peer timeout
	void peer_gather(hipStream_t st, int what, bool poll);
	// Adam on parameters [begin, end) only (data-parallel sharded optimizer: each rank updates its
	// shard of the reduce-scattered gradient, then the fp16 parameters are all-gathered)
	void optimizer_step_range(hipStream_t st, uint64_t begin, uint64_t end);
	float loss(hipStream_t st);
	void inference(hipStream_t st, uint32_t B, const float* input, float* out);
	void set_params_full_precision(const float* host, uint64_t n);
	// snapshot in the reference's msgpack format (Trainer::serialize / deserialize, trainer.h:275-315)
	std::vector<uint8_t> serialize(bool with_optimizer);
	// the same object as JSON text, binaries as {"bytes": [...], "subtype": null} (json serialize(bool))
	std::string serialize_json(bool with_optimizer);
	void deserialize(const void* data, size_t size);
	void mark(hipStream_t st, int phase);  // records phase boundary when timing is enabled
	void profile_end(double* ms, uint32_t n_phases, uint32_t* n_steps);

	// hipGraph replay of the single-GPU training step (the reference Trainer's CUDA graph,
	// trainer.h:163-190, cuda_graph.h:52-178). Opt-in (tcnn_trainer_set_graph). A graph is replayed
	// while every scalar and device pointer the step's kernels read is unchanged (graph_key); any
	// change (batch size, input / target buffers, hyper-parameters, scales, workspace growth) runs
	// the step eagerly and re-captures. The Adam bias-factor table is filled GRAPH_STEPS steps ahead
	// first, so a replayed step carries no step-dependent kernel argument.
	static constexpr uint32_t GRAPH_STEPS = 1u << 20;
	bool use_graph = false;
	struct StepGraph;
	std::unique_ptr<StepGraph> graph;
	uint64_t graph_replays = 0, graph_captures = 0;
	std::vector<uint64_t> graph_key(uint32_t B, const float* input, const float* target) const;
	bool training_step_graph(hipStream_t st, uint32_t B, const float* input, const float* target);
	void set_graph(bool on);
	~TrainerHost();
};

}  // namespace tcnn_amd
