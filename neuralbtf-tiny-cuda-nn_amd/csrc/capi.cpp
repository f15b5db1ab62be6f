// capi.cpp -- extern "C" boundary (include/tcnn_mi355x.h). Exceptions stop here and become return
// codes + tcnn_last_error().
#include "../../include/tcnn_mi355x.h"
#include "debug_api.h"  // test-only diagnostics, not in the product header

#include <algorithm>
#include <cstring>
#include <mutex>

#include "runtime.h"

using namespace tcnn_amd;

namespace {
thread_local std::string g_last_error;
thread_local std::string g_str;

std::mutex g_log_mutex;
tcnn_log_callback_t g_log_cb = nullptr;
void* g_log_user = nullptr;

template <typename F>
int guard(F&& f) {
	try {
		f();
		return 0;
	} catch (const std::exception& e) {
		g_last_error = e.what();
	} catch (...) {
		g_last_error = "unknown C++ exception";
	}
	return 1;
}

template <typename T, typename F>
T* guard_ptr(F&& f) {
	try {
		return f();
	} catch (const std::exception& e) {
		g_last_error = e.what();
	} catch (...) {
		g_last_error = "unknown C++ exception";
	}
	return nullptr;
}

json parse_json(const char* s) {
	if (!s || !*s) return json::object();
	return json::parse(std::string(s));
}

// ---- runtime module (cpp_api.cu:64-140) ----
// What a forward keeps for its backward (the reference's tcnn::Context, cpp_api.cu:84-94). Buffers come
// from a pool the module and its contexts share, so a context may outlive its module, and steady-state
// training allocates nothing. Like the reference's stream arenas, a context's buffer is stream-ordered:
// the backward must run on the forward's stream (or after it).
struct KeepPool {
	std::mutex mu;
	std::vector<std::unique_ptr<DevBuf>> free;
	std::unique_ptr<DevBuf> get() {
		std::lock_guard<std::mutex> lk(mu);
		if (free.empty()) return std::make_unique<DevBuf>();
		auto b = std::move(free.back());
		free.pop_back();
		return b;
	}
	void put(std::unique_ptr<DevBuf> b) {
		std::lock_guard<std::mutex> lk(mu);
		if (free.size() < 4) free.push_back(std::move(b));  // keeps two forwards in flight without allocating
	}
};

struct ModuleCtx {
	virtual ~ModuleCtx() = default;
};

struct NwieCtx : ModuleCtx {
	std::shared_ptr<KeepPool> pool;
	std::unique_ptr<DevBuf> keep;
	int layout = 0;
	const float* in = nullptr;
	const void* params = nullptr;
	~NwieCtx() override {
		if (pool && keep) pool->put(std::move(keep));
	}
};

struct ModuleBase {
	virtual ~ModuleBase() = default;
	virtual void inference(hipStream_t st, uint32_t n, const float* in, void* out, const void* params) = 0;
	virtual std::unique_ptr<ModuleCtx> forward(hipStream_t st, uint32_t n, const float* in, void* out, const void* params, bool prep) = 0;
	virtual void backward(hipStream_t st, const ModuleCtx* ctx, uint32_t n, float* dL_din, const void* dL_dout, void* dL_dparams,
	                      const float* in, const void* out, const void* params) = 0;
	// tcnn_module_backward_scaled specialised by the module (false: the generic scale / backward /
	// divide sequence runs instead)
	virtual bool backward_scaled(hipStream_t, const ModuleCtx*, uint32_t, float*, const void*, void*, const float*, const void*,
	                             const void*, float, bool) {
		return false;
	}
	// object.h:278-288: only encodings that define it (the grid) support second-order gradients
	virtual void backward_backward_input(hipStream_t, uint32_t, const float*, const float*, const void*, void*, void*, float*,
	                                     const void*) {
		throw std::runtime_error("DifferentiableObject::backward_backward_input_impl: not implemented error");
	}
	virtual GridEncodingHost* grid_encoding() { return nullptr; }
	virtual const char* engine() const { return "encoding"; }
	virtual const char* inference_engine() const { return "encoding"; }
	virtual uint32_t n_input_dims() const = 0;
	virtual uint32_t n_output_dims() const = 0;
	virtual uint64_t n_params() const = 0;
	virtual void initialize_params(uint64_t seed, float* params_fp32, float scale) = 0;
	virtual json hyperparams() const = 0;
	virtual std::string name() const = 0;
	std::string scratch;
};

void check_batch(uint32_t n) {
	TCNN_CHECK(n % BATCH_GRANULARITY == 0, "Batch size must be a multiple of " + std::to_string(BATCH_GRANULARITY));
}

struct ModuleNWIE : ModuleBase {
	NetworkHost model;
	StepWorkspace ws;
	DevBuf grad32;
	std::shared_ptr<KeepPool> pool = std::make_shared<KeepPool>();
	ModuleNWIE(uint32_t n_in, uint32_t n_out, const json& enc, const json& net) : model(n_in, n_out, enc, net) {}
	void inference(hipStream_t st, uint32_t n, const float* in, void* out, const void* params) override {
		check_batch(n);
		model.inference(st, ws, n, in, params, out);
	}
	// The context keeps the encoding of this batch in the layout the backward reads, so the backward
	// does not encode again (the fused grid kernel skips its gathers; the tile engine its encoding pass).
	std::unique_ptr<ModuleCtx> forward(hipStream_t st, uint32_t n, const float* in, void* out, const void* params, bool prep) override {
		check_batch(n);
		auto c = std::make_unique<NwieCtx>();
		c->pool = pool;
		if (model.sw.no_forward_keep) {  // A/B switch (read when the module is built): the backward recomputes the forward
			model.inference(st, ws, n, in, params, out);
			c->layout = NetworkHost::KEEP_NONE;
			return c;
		}
		c->keep = pool->get();
		c->layout = model.forward_keep(st, ws, n, in, params, out, prep, *c->keep);
		c->in = in;
		c->params = params;
		return c;
	}
	void backward(hipStream_t st, const ModuleCtx* ctx, uint32_t n, float* dL_din, const void* dL_dout, void* dL_dparams, const float* in,
	              const void*, const void* params) override {
		check_batch(n);
		if (!dL_dparams && !dL_din) return;
		grad32.reserve(n_params() * 4);
		// the kept encoding describes this batch only if the backward sees the forward's input and parameters
		const NwieCtx* c = dynamic_cast<const NwieCtx*>(ctx);
		const bool use = c && c->keep && c->layout != NetworkHost::KEEP_NONE && c->in == in && c->params == params;
		model.fwd_bwd(st, ws, n, in, nullptr, model.n_output_dims, 1.0f, params, dL_dout, nullptr, grad32.as<float>(), nullptr, dL_din,
		              use ? c->keep->p : nullptr, use ? c->layout : NetworkHost::KEEP_NONE);
		if (dL_dparams) launch_cast_f32_f16(st, grad32.as<float>(), dL_dparams, n_params());
	}
	// the torch binding's backward in as few launches as the engine allows: the loss scale folded
	// into the fused kernel's dL/dy load (or one scaling pass for the other engines), the gradient
	// finalised as fp16(fp16(g) / s) in one pass (launch_grad_finalize) instead of a cast and a division
	bool backward_scaled(hipStream_t st, const ModuleCtx* ctx, uint32_t n, float* dL_din, const void* dL_dout, void* dL_dparams,
	                     const float* in, const void*, const void* params, float s, bool dparams_f32) override {
		check_batch(n);
		if (!dL_dparams && !dL_din) return true;
		grad32.reserve(n_params() * 4);
		const NwieCtx* c = dynamic_cast<const NwieCtx*>(ctx);
		const bool use = c && c->keep && c->layout != NetworkHost::KEEP_NONE && c->in == in && c->params == params;
		const void* dout = dL_dout;
		const bool fused = model.fused_ok() && !dL_din;
		model.grad_fin_done = false;
		if (fused) {
			model.ext_dout_scale = s;
			if (dL_dparams) model.grad_fin = GradFinalize{dL_dparams, s, dparams_f32 ? 1 : 0};
		} else {
			const size_t n_out = (size_t)n * model.mlp.padded_output;
			dout_scaled.reserve(n_out * 2);
			launch_scale_f16(st, dL_dout, dout_scaled.p, s, n_out);
			dout = dout_scaled.p;
		}
		try {
			model.fwd_bwd(st, ws, n, in, nullptr, model.n_output_dims, 1.0f, params, dout, nullptr, grad32.as<float>(), nullptr, dL_din,
			              use ? c->keep->p : nullptr, use ? c->layout : NetworkHost::KEEP_NONE);
		} catch (...) {
			model.ext_dout_scale = 1.0f;
			model.grad_fin = {};
			throw;
		}
		model.ext_dout_scale = 1.0f;
		model.grad_fin = {};
		if (dL_din) launch_div_f32(st, dL_din, s, (size_t)n * model.n_input_dims);
		if (dL_dparams && !model.grad_fin_done) launch_grad_finalize(st, grad32.as<float>(), dL_dparams, s, n_params(), dparams_f32);
		return true;
	}
	DevBuf dout_scaled;
	GridEncodingHost* grid_encoding() override { return model.grid; }
	const char* engine() const override { return model.engine(); }
	const char* inference_engine() const override { return model.inference_engine(); }
	uint32_t n_input_dims() const override { return model.n_input_dims; }
	uint32_t n_output_dims() const override { return model.mlp.padded_output; }
	uint64_t n_params() const override { return model.n_params(); }
	void initialize_params(uint64_t seed, float* p, float scale) override {
		Pcg32 rng{seed};
		std::vector<float> host(n_params());
		model.initialize_params(rng, host.data(), scale);
		TCNN_HIP_CHECK(hipMemcpy(p, host.data(), host.size() * 4, hipMemcpyHostToDevice));
	}
	json hyperparams() const override { return model.hyperparams(); }
	std::string name() const override { return "NetworkWithInputEncoding"; }
};

// Parameter-free encodings (OneBlob, Identity) as a module (cpp_api.cu:145-149). Encoding modules take
// any batch size (per-point kernels with bounds checks, like the reference); networks keep the 256 rule.
struct ModuleEncoding : ModuleBase {
	EncodingHost enc;
	ModuleEncoding(uint32_t n_in, const json& j) : enc(n_in, j) {}
	void inference(hipStream_t st, uint32_t n, const float* in, void* out, const void* params) override {
		enc.forward_aos(st, n, in, params, out);
	}
	std::unique_ptr<ModuleCtx> forward(hipStream_t st, uint32_t n, const float* in, void* out, const void* params, bool) override {
		inference(st, n, in, out, params);
		return nullptr;
	}
	void backward(hipStream_t st, const ModuleCtx*, uint32_t n, float* dL_din, const void* dL_dout, void*, const float* in, const void*,
	              const void*) override {
		if (dL_din) enc.backward_input(st, n, in, dL_dout, dL_din);
	}
	uint32_t n_input_dims() const override { return enc.n_dims; }
	uint32_t n_output_dims() const override { return enc.padded_output_width(); }
	uint64_t n_params() const override { return 0; }
	void initialize_params(uint64_t, float*, float) override {}
	json hyperparams() const override { return enc.hyperparams(); }
	std::string name() const override { return enc.kind == EncKind::OneBlob ? "OneBlobEncoding" : "IdentityEncoding"; }
};

struct ModuleGrid : ModuleBase {
	GridEncodingHost grid;
	GridBwdBufs gbw;
	DevBuf grad32;
	ModuleGrid(uint32_t n_in, const json& enc) : grid(n_in, enc) {}
	void inference(hipStream_t st, uint32_t n, const float* in, void* out, const void* params) override {
		const uint32_t W = grid.padded_output_width();
		if (grid.n_to_pad) TCNN_HIP_CHECK(hipMemsetAsync(out, 0, (size_t)n * W * 2, st));
		launch_grid_fwd(st, grid.desc.n_pos_dims, grid.desc.n_features_per_level, grid.desc.hash_type, n, grid.desc.n_levels,
		                in, grid.desc.n_pos_dims, params, out, false, W, grid.dev_levels(), grid.hash_grid(), grid.desc.interp, grid.opts());
	}
	std::unique_ptr<ModuleCtx> forward(hipStream_t st, uint32_t n, const float* in, void* out, const void* params, bool prep) override {
		(void)prep;  // dy/dx is recomputed in backward (launch_grid_bwd_input), nothing to keep
		inference(st, n, in, out, params);
		return nullptr;
	}
	void backward(hipStream_t st, const ModuleCtx*, uint32_t n, float* dL_din, const void* dL_dout, void* dL_dparams, const float* in,
	              const void*, const void* params) override {
		if (dL_din)
			launch_grid_bwd_input(st, grid.desc.n_pos_dims, grid.desc.n_features_per_level, grid.desc.hash_type, n, grid.desc.n_levels, in,
			                      grid.desc.n_pos_dims, params, dL_dout, 2, grid.padded_output_width(), dL_din, grid.desc.n_pos_dims,
			                      grid.dev_levels(), grid.hash_grid(), grid.desc.interp, grid.opts());
		if (!dL_dparams) return;
		grad32.reserve((size_t)grid.n_params * 4);
		grid.backward(st, gbw, n, in, grid.desc.n_pos_dims, dL_dout, 2, grid.padded_output_width(), grad32.as<float>());
		launch_cast_f32_f16(st, grad32.as<float>(), dL_dparams, grid.n_params);
	}
	void backward_backward_input(hipStream_t st, uint32_t n, const float* dL_ddLdin, const float* in, const void* dL_dout,
	                             void* dL_dparams, void* dL_ddLdout, float* dL_din, const void* params) override {
		if (!dL_ddLdout && !dL_dparams) return;  // grid.h:913-915
		TCNN_CHECK(params, "backward_backward_input needs the grid parameters");
		if (dL_dparams) {
			grad32.reserve((size_t)grid.n_params * 4);
			TCNN_HIP_CHECK(hipMemsetAsync(grad32.p, 0, (size_t)grid.n_params * 4, st));  // GradientMode::Overwrite
		}
		const uint32_t W = grid.padded_output_width();
		launch_grid_bwd_bwd(st, grid.desc.n_pos_dims, grid.desc.n_features_per_level, grid.desc.hash_type, n, grid.desc.n_levels, in,
		                    grid.desc.n_pos_dims, params, dL_ddLdin, dL_dout, W, dL_dparams ? grad32.as<float>() : nullptr, dL_ddLdout, W,
		                    dL_din, grid.dev_levels(), grid.hash_grid(), grid.desc.interp, grid.opts());
		if (dL_dparams) launch_cast_f32_f16(st, grad32.as<float>(), dL_dparams, grid.n_params);
	}
	GridEncodingHost* grid_encoding() override { return &grid; }
	uint32_t n_input_dims() const override { return grid.desc.n_pos_dims; }
	uint32_t n_output_dims() const override { return grid.padded_output_width(); }
	uint64_t n_params() const override { return grid.n_params; }
	void initialize_params(uint64_t seed, float* p, float scale) override {
		Pcg32 rng{seed};
		std::vector<float> host(n_params());
		grid.initialize_params(rng, host.data(), scale);
		TCNN_HIP_CHECK(hipMemcpy(p, host.data(), host.size() * 4, hipMemcpyHostToDevice));
	}
	json hyperparams() const override { return grid.hyperparams(); }
	std::string name() const override { return "GridEncoding"; }
};
}  // namespace

struct tcnn_module {
	std::unique_ptr<ModuleBase> m;
	DevBuf dout_scaled, dparams16;  // tcnn_module_backward_scaled's temporaries
};
struct tcnn_context {
	uint32_t n = 0;
	std::unique_ptr<ModuleCtx> impl;  // what the forward kept (nullptr: nothing)
};
struct tcnn_trainer {
	std::unique_ptr<TrainerHost> t;
};
struct tcnn_dp_comm {
	std::unique_ptr<DpComm> c;
};

extern "C" {

const char* tcnn_last_error(void) { return g_last_error.c_str(); }
const char* tcnn_version(void) { return "tcnn-mi355x 0.1 (gfx950)"; }
uint32_t tcnn_batch_size_granularity(void) { return BATCH_GRANULARITY; }
int tcnn_cuda_device(void) {
	int d = -1;
	if (hipGetDevice(&d) != hipSuccess) return -1;
	return d;
}
int tcnn_set_cuda_device(int device) {
	return guard([&] { TCNN_HIP_CHECK(hipSetDevice(device)); });
}
void tcnn_free_temporary_memory(void) {  // free_all_gpu_memory_arenas (gpu_memory.h:751-754)
	try {
		tcnn_amd::workspace_arena_free_all();
	} catch (...) {
	}
}
int tcnn_has_networks(void) { return 1; }

int tcnn_generate_random_logistic(void* stream, uint64_t* rng_state, uint64_t* rng_inc, uint64_t n, float* out, float mean, float stddev) {
	return guard([&] {
		TCNN_CHECK(rng_state && rng_inc, "generate_random_logistic: rng state missing");
		launch_generate_logistic((hipStream_t)stream, n, *rng_state, *rng_inc, out, mean, stddev);
		Pcg32 r;
		r.state = *rng_state;
		r.inc = *rng_inc;
		r.advance((int64_t)n);  // random.h:64
		*rng_state = r.state;
	});
}
int tcnn_generate_random_uniform(void* stream, uint64_t* rng_state, uint64_t* rng_inc, uint64_t n, float* out, float lower, float upper) {
	return guard([&] {
		TCNN_CHECK(rng_state && rng_inc, "generate_random_uniform: rng state missing");
		launch_generate_uniform((hipStream_t)stream, n, *rng_state, *rng_inc, out, lower, upper);
		Pcg32 r;
		r.state = *rng_state;
		r.inc = *rng_inc;
		r.advance((int64_t)n);  // rng.advance(n_elements), random.h:64
		*rng_state = r.state;
	});
}

void tcnn_set_log_callback(tcnn_log_callback_t cb, void* user) {
	std::lock_guard<std::mutex> lk(g_log_mutex);
	g_log_cb = cb;
	g_log_user = user;
}
float tcnn_default_loss_scale(int precision) { return precision == TCNN_PRECISION_FP32 ? 1.0f : 128.0f; }
int tcnn_preferred_precision(void) { return TCNN_PRECISION_FP16; }

tcnn_module* tcnn_create_network_with_input_encoding(uint32_t n_in, uint32_t n_out, const char* enc, const char* net) {
	return guard_ptr<tcnn_module>([&] {
		auto* r = new tcnn_module;
		r->m = std::make_unique<ModuleNWIE>(n_in, n_out, parse_json(enc), parse_json(net));
		return r;
	});
}

// create_network = Identity encoding + network (cpp_api.cu:151-153)
tcnn_module* tcnn_create_network(uint32_t n_in, uint32_t n_out, const char* net) {
	return guard_ptr<tcnn_module>([&] {
		auto* r = new tcnn_module;
		r->m = std::make_unique<ModuleNWIE>(n_in, n_out, json{{"otype", "Identity"}}, parse_json(net));
		return r;
	});
}

tcnn_module* tcnn_create_encoding(uint32_t n_in, const char* enc, int precision) {
	return guard_ptr<tcnn_module>([&] {
		TCNN_CHECK(precision == TCNN_PRECISION_FP16, "create_encoding: only Fp16 precision is implemented by the MI355X engine");
		json j = parse_json(enc);
		const std::string ot = j.is_object() && j.find("otype") != j.end() ? j["otype"].get<std::string>() : "OneBlob";
		TCNN_CHECK(EncodingHost::known(ot), "Encoding '" + ot + "' is not implemented by the MI355X engine yet");
		auto* r = new tcnn_module;
		if (ieq(ot, "OneBlob") || ieq(ot, "Identity")) r->m = std::make_unique<ModuleEncoding>(n_in, j);
		else r->m = std::make_unique<ModuleGrid>(n_in, j);
		return r;
	});
}

void tcnn_module_destroy(tcnn_module* m) { delete m; }

int tcnn_module_inference(tcnn_module* m, void* stream, uint32_t n, const float* in, void* out, const void* params) {
	if (n == 0) return 0;  // empty batch: nothing to do (every kernel would be a zero-size launch)
	return guard([&] { m->m->inference((hipStream_t)stream, n, in, out, params); });
}

tcnn_context* tcnn_module_forward(tcnn_module* m, void* stream, uint32_t n, const float* in, void* out, const void* params, int prep) {
	return guard_ptr<tcnn_context>([&] {
		auto* c = new tcnn_context;
		c->n = n;
		if (n) c->impl = m->m->forward((hipStream_t)stream, n, in, out, params, prep != 0);
		return c;
	});
}

int tcnn_module_backward(tcnn_module* m, void* stream, const tcnn_context* ctx, uint32_t n, float* dL_din, const void* dL_dout,
                         void* dL_dparams, const float* in, const void* out, const void* params) {
	return guard([&] {
		TCNN_CHECK(ctx != nullptr, "backward: null context");
		if (n == 0) {  // empty batch: Overwrite-mode gradients are all zero
			if (dL_dparams) TCNN_HIP_CHECK(hipMemsetAsync(dL_dparams, 0, m->m->n_params() * 2, (hipStream_t)stream));
			return;
		}
		TCNN_CHECK(ctx->n == n, "backward: batch size differs from the forward's");
		m->m->backward((hipStream_t)stream, ctx->impl.get(), n, dL_din, dL_dout, dL_dparams, in, out, params);
	});
}

int tcnn_module_backward_scaled(tcnn_module* m, void* stream, const tcnn_context* ctx, uint32_t n, float* dL_din, const void* dL_dout,
                                void* dL_dparams, const float* in, const void* out, const void* params, float loss_scale,
                                int dparams_fp32) {
	return guard([&] {
		TCNN_CHECK(ctx != nullptr, "backward: null context");
		TCNN_CHECK(loss_scale != 0.0f, "backward: loss scale must be nonzero");
		const hipStream_t st = (hipStream_t)stream;
		const uint64_t np = m->m->n_params();
		if (n == 0) {
			if (dL_dparams) TCNN_HIP_CHECK(hipMemsetAsync(dL_dparams, 0, np * (dparams_fp32 ? 4 : 2), st));
			return;
		}
		TCNN_CHECK(ctx->n == n, "backward: batch size differs from the forward's");
		if (m->m->backward_scaled(st, ctx->impl.get(), n, dL_din, dL_dout, dL_dparams, in, out, params, loss_scale, dparams_fp32 != 0))
			return;
		const size_t n_out = (size_t)n * m->m->n_output_dims();
		m->dout_scaled.reserve(n_out * 2);
		launch_scale_f16(st, dL_dout, m->dout_scaled.p, loss_scale, n_out);  // modules.py:135 doutput * loss_scale
		void* g16 = dL_dparams;
		if (dL_dparams && dparams_fp32) {
			m->dparams16.reserve(np * 2);
			g16 = m->dparams16.p;
		}
		m->m->backward(st, ctx->impl.get(), n, dL_din, m->dout_scaled.p, g16, in, out, params);
		if (dL_din) launch_div_f32(st, dL_din, loss_scale, (size_t)n * m->m->n_input_dims());  // modules.py:137
		if (dL_dparams) launch_div_f16(st, g16, dL_dparams, loss_scale, np, dparams_fp32 != 0);  // modules.py:138
	});
}

int tcnn_module_backward_backward_input(tcnn_module* m, void* stream, const tcnn_context* ctx, uint32_t n, const float* dL_ddLdin,
                                        const float* in, const void* dL_dout, void* dL_dparams, void* dL_ddLdout, float* dL_din,
                                        const void* params) {
	return guard([&] {
		TCNN_CHECK(ctx != nullptr, "backward_backward_input: null context");
		if (n == 0) {
			if (dL_dparams) TCNN_HIP_CHECK(hipMemsetAsync(dL_dparams, 0, m->m->n_params() * 2, (hipStream_t)stream));
			return;
		}
		m->m->backward_backward_input((hipStream_t)stream, n, dL_ddLdin, in, dL_dout, dL_dparams, dL_ddLdout, dL_din, params);
	});
}

void tcnn_context_destroy(tcnn_context* c) { delete c; }

static GridEncodingHost& module_grid(tcnn_module* m) {
	GridEncodingHost* g = m->m->grid_encoding();
	TCNN_CHECK(g != nullptr, "module has no grid encoding");
	return *g;
}
int tcnn_module_set_max_level(tcnn_module* m, float max_level) {
	return guard([&] { module_grid(m).max_level = max_level; });
}
float tcnn_module_max_level(tcnn_module* m) {
	float v = -1.0f;
	guard([&] { v = module_grid(m).max_level; });
	return v;
}
int tcnn_module_set_max_level_gpu(tcnn_module* m, const float* max_level_per_point) {
	return guard([&] { module_grid(m).max_level_gpu = max_level_per_point; });
}
uint32_t tcnn_module_n_input_dims(const tcnn_module* m) { return m->m->n_input_dims(); }
uint32_t tcnn_module_n_output_dims(const tcnn_module* m) { return m->m->n_output_dims(); }
uint64_t tcnn_module_n_params(const tcnn_module* m) { return m->m->n_params(); }
int tcnn_module_param_precision(const tcnn_module*) { return TCNN_PRECISION_FP16; }
int tcnn_module_output_precision(const tcnn_module*) { return TCNN_PRECISION_FP16; }
int tcnn_module_initialize_params(tcnn_module* m, uint64_t seed, float* p, float scale) {
	return guard([&] { m->m->initialize_params(seed, p, scale); });
}
const char* tcnn_module_hyperparams(tcnn_module* m) {
	m->m->scratch = m->m->hyperparams().dump();
	return m->m->scratch.c_str();
}
const char* tcnn_module_name(tcnn_module* m) {
	m->m->scratch = m->m->name();
	return m->m->scratch.c_str();
}

tcnn_trainer* tcnn_trainer_create(uint32_t n_in, uint32_t n_out, const char* cfg, uint32_t seed) {
	return guard_ptr<tcnn_trainer>([&] {
		auto* r = new tcnn_trainer;
		r->t = std::make_unique<TrainerHost>(n_in, n_out, parse_json(cfg), seed);
		return r;
	});
}
void tcnn_trainer_destroy(tcnn_trainer* t) { delete t; }
int tcnn_trainer_training_step(tcnn_trainer* t, void* stream, uint32_t n, const float* in, const float* target, int run_opt) {
	return guard([&] {
		TCNN_CHECK(n > 0, "training_step: empty batch");
		t->t->training_step((hipStream_t)stream, n, in, target, run_opt != 0);
	});
}
int tcnn_trainer_training_step_part(tcnn_trainer* t, void* stream, uint32_t n, const float* in, const float* target, int part) {
	return guard([&] { t->t->training_step_part((hipStream_t)stream, n, in, target, part); });
}
int tcnn_trainer_optimizer_step(tcnn_trainer* t, void* stream) {
	return guard([&] { t->t->optimizer_step((hipStream_t)stream); });
}
void* tcnn_workspace_allocate(void* stream, uint64_t n_bytes) {
	void* p = nullptr;
	guard([&] { p = workspace_allocate((hipStream_t)stream, n_bytes); });
	return p;
}
int tcnn_workspace_free(void* stream, void* ptr) {
	return guard([&] { workspace_free((hipStream_t)stream, ptr); });
}
int tcnn_free_workspace_arena(void* stream) {
	return guard([&] { workspace_arena_free((hipStream_t)stream); });
}
int tcnn_workspace_arena_info(void* stream, uint64_t* mapped_bytes, int* virtual_memory) {
	return guard([&] { workspace_arena_info((hipStream_t)stream, mapped_bytes, virtual_memory); });
}

struct tcnn_trainer_context {
	std::unique_ptr<TrainerFwdCtx> c;
};
tcnn_trainer_context* tcnn_trainer_forward(tcnn_trainer* t, void* stream, uint32_t n, const float* in, const float* target, const float* pdf,
                                           const void* ext, int prep) {
	tcnn_trainer_context* r = nullptr;
	const int rc = guard([&] {
		TCNN_CHECK(n > 0, "forward: empty batch");
		auto c = t->t->forward((hipStream_t)stream, n, in, target, pdf, ext, prep != 0);
		r = new tcnn_trainer_context{std::move(c)};
	});
	return rc == 0 ? r : nullptr;
}
tcnn_trainer_context* tcnn_trainer_forward_perturbed(tcnn_trainer* t, void* stream, uint32_t n, const float* in, const float* target,
                                                     const float* pdf, const float* perturbation, int prep) {
	tcnn_trainer_context* r = nullptr;
	const int rc = guard([&] {
		TCNN_CHECK(n > 0, "forward: empty batch");
		TCNN_CHECK(target != nullptr, "forward_perturbed: a target is required");
		auto c = t->t->forward((hipStream_t)stream, n, in, target, pdf, nullptr, prep != 0, perturbation);
		r = new tcnn_trainer_context{std::move(c)};
	});
	return rc == 0 ? r : nullptr;
}
int tcnn_trainer_backward(tcnn_trainer* t, void* stream, const tcnn_trainer_context* ctx, uint32_t n, const float* in, float* dL_din,
                          int gradient_mode) {
	return guard([&] {
		TCNN_CHECK(ctx != nullptr, "backward: null context");
		TCNN_CHECK(gradient_mode >= 0 && gradient_mode <= 2, "backward: gradient_mode must be 0 (Overwrite), 1 (Accumulate) or 2 (Ignore)");
		t->t->backward((hipStream_t)stream, *ctx->c, n, in, dL_din, gradient_mode);
	});
}
float tcnn_trainer_context_loss(tcnn_trainer* t, void* stream, const tcnn_trainer_context* ctx) {
	float v = -1.0f;
	guard([&] {
		TCNN_CHECK(ctx != nullptr, "loss: null context");
		v = t->t->ctx_loss((hipStream_t)stream, *ctx->c);
	});
	return v;
}
const void* tcnn_trainer_context_output(const tcnn_trainer_context* ctx) { return ctx ? ctx->c->out16.p : nullptr; }
const void* tcnn_trainer_context_doutput(const tcnn_trainer_context* ctx) { return ctx ? ctx->c->dLdy() : nullptr; }
void tcnn_trainer_context_destroy(tcnn_trainer_context* ctx) { delete ctx; }
uint32_t tcnn_trainer_padded_output_width(const tcnn_trainer* t) { return t->t->model->mlp.padded_output; }
int tcnn_trainer_optimizer_step_range(tcnn_trainer* t, void* stream, uint64_t begin, uint64_t end) {
	return guard([&] { t->t->optimizer_step_range((hipStream_t)stream, begin, end); });
}
int tcnn_dp_unique_id(void* id) {
	return guard([&] { dp_unique_id(id); });
}
tcnn_dp_comm* tcnn_dp_comm_create(const void* id, int nranks, int rank) {
	return guard_ptr<tcnn_dp_comm>([&] {
		auto* r = new tcnn_dp_comm;
		r->c = std::make_unique<DpComm>(id, nranks, rank);
		return r;
	});
}
void tcnn_dp_comm_destroy(tcnn_dp_comm* c) { delete c; }
int tcnn_trainer_set_dp(tcnn_trainer* t, tcnn_dp_comm* c, int sharded) {
	return guard([&] { t->t->set_dp(c ? c->c.get() : nullptr, sharded != 0); });
}
uint64_t tcnn_dp_peer_blob_bytes(void) { return tcnn_amd::dp_peer_blob_bytes(); }
int tcnn_trainer_dp_peer_export(tcnn_trainer* t, int nranks, int rank, void* blob) {
	return guard([&] { t->t->dp_peer_export(nranks, rank, blob); });
}
int tcnn_trainer_dp_peer_attach(tcnn_trainer* t, const void* blobs) {
	return guard([&] { t->t->dp_peer_attach(blobs); });
}
int tcnn_trainer_dp_peer_detach(tcnn_trainer* t) {
	return guard([&] { t->t->dp_peer_detach(); });
}
int tcnn_trainer_dp_peer_set_timeout(tcnn_trainer* t, double seconds) {
	return guard([&] { t->t->dp_peer_set_timeout(seconds); });
}
int tcnn_debug_peer_loopback(tcnn_trainer* t, int nranks) {
	return guard([&] { t->t->dp_peer_loopback(nranks); });
}
int tcnn_trainer_dp_peer_abandon(tcnn_trainer* t) {
	return guard([&] { t->t->dp_peer_abandon(); });
}
int tcnn_trainer_dp_gather_state(tcnn_trainer* t, void* stream) {
	return guard([&] { t->t->dp_gather_state((hipStream_t)stream); });
}
float tcnn_trainer_loss(tcnn_trainer* t, void* stream) {
	float v = -1.0f;
	if (guard([&] { v = t->t->loss((hipStream_t)stream); }) != 0) return -1.0f;
	return v;
}
const float* tcnn_trainer_loss_device(tcnn_trainer* t) { return t->t->d_loss.as<float>(); }
int tcnn_trainer_inference(tcnn_trainer* t, void* stream, uint32_t n, const float* in, float* out) {
	return guard([&] {
		if (n) t->t->inference((hipStream_t)stream, n, in, out);
	});
}
uint64_t tcnn_trainer_n_params(const tcnn_trainer* t) { return t->t->n_params; }
uint64_t tcnn_trainer_n_network_params(const tcnn_trainer* t) { return t->t->n_mlp; }
float* tcnn_trainer_params_fp32(tcnn_trainer* t) { return t->t->w32.as<float>(); }
void* tcnn_trainer_params(tcnn_trainer* t) { return t->t->w16.p; }
void* tcnn_trainer_param_gradients(tcnn_trainer* t) { return t->t->g16.p; }
float* tcnn_trainer_gradients_fp32(tcnn_trainer* t) { return t->t->g32.as<float>(); }
int tcnn_trainer_optimizer_state(tcnn_trainer* t, float** m1, float** m2, uint32_t** steps) {
	if (m1) *m1 = t->t->m1.as<float>();
	if (m2) *m2 = t->t->m2.as<float>();
	if (steps) *steps = t->t->steps.as<uint32_t>();
	return 0;
}
int tcnn_trainer_set_gradient_scale(tcnn_trainer* t, float s) {
	TrainerHost& h = *t->t;
	h.grad_scale_user = s;
	h.grad_scale = s / (float)h.dp_nranks();  // the RCCL communicator's or the peer exchange's N
	return 0;
}
int tcnn_trainer_set_loss_scale(tcnn_trainer* t, float loss_scale) {
	return guard([&] {
		TCNN_CHECK(loss_scale > 0.0f && std::isfinite(loss_scale), "set_loss_scale: the loss scale must be positive and finite");
		t->t->loss_scale = loss_scale;
	});
}
int tcnn_trainer_set_graph(tcnn_trainer* t, int on) {
	return guard([&] { t->t->set_graph(on != 0); });
}
int tcnn_trainer_graph_stats(const tcnn_trainer* t, uint64_t* captures, uint64_t* replays) {
	if (captures) *captures = t->t->graph_captures;
	if (replays) *replays = t->t->graph_replays;
	return 0;
}
int tcnn_trainer_serialize(tcnn_trainer* t, int with_optimizer, void* buf, uint64_t capacity, uint64_t* size) {
	return guard([&] {
		const std::vector<uint8_t> b = t->t->serialize(with_optimizer != 0);
		if (size) *size = b.size();
		if (buf) {
			TCNN_CHECK(capacity >= b.size(), "tcnn_trainer_serialize: buffer too small");
			std::memcpy(buf, b.data(), b.size());
		}
	});
}
int tcnn_trainer_serialize_json(tcnn_trainer* t, int with_optimizer, char* buf, uint64_t capacity, uint64_t* size) {
	return guard([&] {
		const std::string j = t->t->serialize_json(with_optimizer != 0);
		if (size) *size = j.size() + 1;
		if (buf) {
			TCNN_CHECK(capacity >= j.size() + 1, "tcnn_trainer_serialize_json: buffer too small");
			std::memcpy(buf, j.c_str(), j.size() + 1);
		}
	});
}
int tcnn_trainer_deserialize(tcnn_trainer* t, const void* buf, uint64_t size) {
	return guard([&] { t->t->deserialize(buf, (size_t)size); });
}
int tcnn_trainer_set_params_full_precision(tcnn_trainer* t, const float* host, uint64_t n) {
	return guard([&] { t->t->set_params_full_precision(host, n); });
}
uint32_t tcnn_trainer_optimizer_step_count(const tcnn_trainer* t) { return t->t->adam_step; }
int tcnn_trainer_update_hyperparams(tcnn_trainer* t, const char* params_json) {
	return guard([&] {
		const json p = json::parse(params_json);
		if (p.count("optimizer")) t->t->adam.update(p["optimizer"]);  // Trainer::update_hyperparams, trainer.h:213-216
		// the reference forwards "loss" to Loss::update_hyperparams, which holds no hyperparameters
		// (relative_l2.h, l2.h): the loss type is fixed at construction there too -- say so instead of
		// ignoring a request to change it
		if (p.count("loss") && p["loss"].is_object() && p["loss"].count("otype")) {
			const std::string o = p["loss"]["otype"].get<std::string>();
			TCNN_CHECK(ieq(o, t->t->loss_otype), "update_hyperparams: the loss type is fixed at construction ('" + t->t->loss_otype +
			                                         "'), cannot change it to '" + o + "'");
		}
	});
}
const char* tcnn_trainer_hyperparams(tcnn_trainer* t) {
	g_str.clear();
	if (guard([&] {
		    json h = json::object();
		    h["optimizer"] = t->t->adam.hyperparams();
		    h["loss"] = json::object();
		    h["loss"]["otype"] = t->t->loss_otype;
		    g_str = h.dump();
	    }) != 0)
		return nullptr;
	return g_str.c_str();
}
int tcnn_trainer_initialize_params_rng(tcnn_trainer* t, uint64_t* state, uint64_t inc) {
	return guard([&] {
		TCNN_CHECK(state != nullptr, "initialize_params_rng: null state");
		Pcg32 rng;
		rng.state = *state;
		rng.inc = inc;
		t->t->initialize_params_rng(rng);
		*state = rng.state;
	});
}
int tcnn_trainer_initialize_params(tcnn_trainer* t, uint32_t seed) {
	return guard([&] { t->t->initialize_params(seed); });
}
const char* tcnn_trainer_engine(const tcnn_trainer* t) { return t->t->model->engine(); }
const char* tcnn_trainer_inference_engine(const tcnn_trainer* t) { return t->t->model->inference_engine(); }
const char* tcnn_module_engine(const tcnn_module* m) { return m->m->engine(); }
const char* tcnn_module_inference_engine(const tcnn_module* m) { return m->m->inference_engine(); }
int tcnn_trainer_set_max_level(tcnn_trainer* t, float max_level) {
	return guard([&] {
		TCNN_CHECK(t->t->model->grid != nullptr, "trainer model has no grid encoding");
		t->t->model->grid->max_level = max_level;
	});
}

int tcnn_trainer_profile_begin(tcnn_trainer* t) { return tcnn_trainer_profile_begin_sampled(t, 1); }
int tcnn_trainer_profile_begin_sampled(tcnn_trainer* t, uint32_t every) {
	return guard([&] {
		t->t->timer.reset();
		t->t->timer.every = every ? every : 1;
		t->t->timer.counter = 0;
		t->t->timer.enabled = true;
	});
}
int tcnn_trainer_profile_end(tcnn_trainer* t, double* ms, uint32_t n_phases, uint32_t* n_steps) {
	return guard([&] { t->t->profile_end(ms, n_phases, n_steps); });
}

int tcnn_debug_fused_phase_cycles(tcnn_trainer* t, void* stream, uint32_t n, const float* input, const float* target,
                                  uint64_t* host_cycles8) {
	return guard([&] {
		auto& tr = *t->t;
		auto& m = *tr.model;
		TCNN_CHECK(m.mlp.width == 64 && m.mlp.n_input == 32 && m.mlp.n_hidden_layers == 2 && m.grid->desc.n_pos_dims == 2,
		           "phase profile: config_hash shape only");
		hipStream_t st = (hipStream_t)stream;
		// run one normal step first so the workspace is sized
		tr.training_step(st, n, input, target, false);
		const uint32_t nb = fused_train_n_blocks(64, 32, 2, 2, tr.n_output_dims, false, n);
		const size_t WV = fused_train_waves();  // waves per workgroup of the fused kernel
		DevBuf prof;
		prof.reserve((size_t)nb * WV * 16 * 8);
		TCNN_HIP_CHECK(hipMemsetAsync(prof.p, 0, (size_t)nb * WV * 16 * 8, st));
		launch_fused_train_profile(st, n, tr.n_output_dims, tr.w16.p, (const uint8_t*)tr.w16.p + tr.n_mlp * 2, input, target,
		                           tr.ws.dLdenc.p, tr.ws.wgrad_partial.as<float>(), tr.ws.loss_partial.as<float>(),
		                           m.grid->dev_levels(), nb, tr.ws.wimage.p, prof.as<unsigned long long>());
		std::vector<unsigned long long> h((size_t)nb * WV * 16);
		TCNN_HIP_CHECK(hipMemcpyAsync(h.data(), prof.p, h.size() * 8, hipMemcpyDeviceToHost, st));
		TCNN_HIP_CHECK(hipStreamSynchronize(st));
		for (int k = 0; k < 16; ++k) {
			unsigned long long sum = 0;
			for (size_t w = 0; w < (size_t)nb * WV; ++w) sum += h[w * 16 + k];
			host_cycles8[k] = sum;
		}
	});
}

int tcnn_debug_hfma(void* stream, const void* a, const void* b, const void* c, void* out, uint32_t n_pairs) {
	return guard([&] { launch_probe_hfma((hipStream_t)stream, a, b, c, out, n_pairs); });
}

int tcnn_debug_probe(void* stream, float* mfma_out, int16_t* tr_out) {
	return guard([&] { launch_probe((hipStream_t)stream, mfma_out, tr_out); });
}

}  // extern "C"

namespace tcnn_amd {
void log_msg(LogSeverity s, const std::string& msg) {
	std::lock_guard<std::mutex> lk(g_log_mutex);
	if (g_log_cb) g_log_cb((int)s, msg.c_str(), g_log_user);
}
}  // namespace tcnn_amd
