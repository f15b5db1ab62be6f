// tiny-cuda-nn/cpp_api.h -- source-compatible `tcnn::cpp` runtime API (reference
// include/tiny-cuda-nn/cpp_api.h:50-117) over the MI355X engine's C-ABI (include/tcnn_mi355x.h).
//
// Header-only: a caller written against the reference's header (the NeuralBTF / torch-extension
// side) compiles unchanged against this one and links libtcnn_mi355x.so. Streams are hipStream_t
// (the reference's cudaStream_t); errors come back as std::runtime_error with tcnn_last_error(),
// as the reference's CHECK_THROW does.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>

#include "common.h"  // tcnn::Context, json, the C-ABI

namespace tcnn { namespace cpp {

enum class LogSeverity { Info, Debug, Warning, Error, Success };

using json = nlohmann::json;

namespace detail {
inline void check(int rc) {
	if (rc != 0) throw std::runtime_error(tcnn_last_error());
}
template <class T>
inline T* check_ptr(T* p) {
	if (!p) throw std::runtime_error(tcnn_last_error());
	return p;
}
struct NativeContext : tcnn::Context {
	tcnn_context* h;
	explicit NativeContext(tcnn_context* c) : h(c) {}
	~NativeContext() override { tcnn_context_destroy(h); }
};
}  // namespace detail

inline uint32_t batch_size_granularity() { return tcnn_batch_size_granularity(); }
inline int cuda_device() { return tcnn_cuda_device(); }
inline void set_cuda_device(int device) { detail::check(tcnn_set_cuda_device(device)); }
inline void free_temporary_memory() { tcnn_free_temporary_memory(); }
inline bool has_networks() { return tcnn_has_networks() != 0; }

enum class Precision { Fp32, Fp16 };

inline float default_loss_scale(Precision p) {
	return tcnn_default_loss_scale(p == Precision::Fp16 ? TCNN_PRECISION_FP16 : TCNN_PRECISION_FP32);
}
inline Precision preferred_precision() {
	return tcnn_preferred_precision() == TCNN_PRECISION_FP16 ? Precision::Fp16 : Precision::Fp32;
}
// cpp_api.cu:61-63: the engine's log messages (grid level table, trainer init, engine fallbacks)
// reach `callback`; an empty function removes it.
namespace detail {
inline std::function<void(LogSeverity, const std::string&)>& log_fn() {
	static std::function<void(LogSeverity, const std::string&)> f;
	return f;
}
inline void log_trampoline(int severity, const char* msg, void*) {
	if (log_fn()) log_fn()((LogSeverity)severity, msg);
}
}  // namespace detail
inline void set_log_callback(const std::function<void(LogSeverity, const std::string&)>& callback) {
	detail::log_fn() = callback;
	tcnn_set_log_callback(callback ? &detail::log_trampoline : nullptr, nullptr);
}

struct Context {  // cpp_api.h:82-84
	std::unique_ptr<tcnn::Context> ctx;
};

class Module {  // cpp_api.h:86-112
public:
	Module(Precision param_precision, Precision output_precision)
	    : m_param_precision{param_precision}, m_output_precision{output_precision} {}
	virtual ~Module() {}

	virtual void inference(hipStream_t stream, uint32_t n_elements, const float* input, void* output, void* params) = 0;
	virtual Context forward(hipStream_t stream, uint32_t n_elements, const float* input, void* output, void* params,
	                        bool prepare_input_gradients) = 0;
	virtual void backward(hipStream_t stream, const Context& ctx, uint32_t n_elements, float* dL_dinput, const void* dL_doutput,
	                      void* dL_dparams, const float* input, const void* output, const void* params) = 0;
	virtual void backward_backward_input(hipStream_t stream, const Context& ctx, uint32_t n_elements, const float* dL_ddLdinput,
	                                     const float* input, const void* dL_doutput, void* dL_dparams, void* dL_ddLdoutput,
	                                     float* dL_dinput, const void* params) = 0;

	virtual uint32_t n_input_dims() const = 0;
	virtual uint32_t n_output_dims() const = 0;
	Precision output_precision() const { return m_output_precision; }

	virtual size_t n_params() const = 0;
	Precision param_precision() const { return m_param_precision; }

	virtual void initialize_params(size_t seed, float* params_full_precision, float scale = 1.0f) = 0;

	virtual json hyperparams() const = 0;
	virtual std::string name() const = 0;

private:
	Precision m_param_precision;
	Precision m_output_precision;
};

namespace detail {
// The one implementation: every factory returns a NativeModule over a C-ABI handle.
class NativeModule : public Module {
public:
	explicit NativeModule(tcnn_module* h)
	    : Module(tcnn_module_param_precision(check_ptr(h)) == TCNN_PRECISION_FP16 ? Precision::Fp16 : Precision::Fp32,
	             tcnn_module_output_precision(h) == TCNN_PRECISION_FP16 ? Precision::Fp16 : Precision::Fp32),
	      m_h(h) {}
	~NativeModule() override { tcnn_module_destroy(m_h); }

	void inference(hipStream_t stream, uint32_t n, const float* input, void* output, void* params) override {
		check(tcnn_module_inference(m_h, stream, n, input, output, params));
	}
	Context forward(hipStream_t stream, uint32_t n, const float* input, void* output, void* params, bool prep) override {
		tcnn_context* c = check_ptr(tcnn_module_forward(m_h, stream, n, input, output, params, prep ? 1 : 0));
		return Context{std::make_unique<NativeContext>(c)};
	}
	void backward(hipStream_t stream, const Context& ctx, uint32_t n, float* dL_dinput, const void* dL_doutput, void* dL_dparams,
	              const float* input, const void* output, const void* params) override {
		check(tcnn_module_backward(m_h, stream, native(ctx), n, dL_dinput, dL_doutput, dL_dparams, input, output, params));
	}
	void backward_backward_input(hipStream_t stream, const Context& ctx, uint32_t n, const float* dL_ddLdinput, const float* input,
	                             const void* dL_doutput, void* dL_dparams, void* dL_ddLdoutput, float* dL_dinput,
	                             const void* params) override {
		check(tcnn_module_backward_backward_input(m_h, stream, native(ctx), n, dL_ddLdinput, input, dL_doutput, dL_dparams,
		                                          dL_ddLdoutput, dL_dinput, params));
	}
	uint32_t n_input_dims() const override { return tcnn_module_n_input_dims(m_h); }
	uint32_t n_output_dims() const override { return tcnn_module_n_output_dims(m_h); }
	size_t n_params() const override { return (size_t)tcnn_module_n_params(m_h); }
	void initialize_params(size_t seed, float* params_full_precision, float scale = 1.0f) override {
		check(tcnn_module_initialize_params(m_h, (uint64_t)seed, params_full_precision, scale));
	}
	json hyperparams() const override { return json::parse(tcnn_module_hyperparams(m_h)); }
	std::string name() const override { return tcnn_module_name(m_h); }
	tcnn_module* handle() const { return m_h; }

private:
	static const tcnn_context* native(const Context& ctx) {
		const auto* c = dynamic_cast<const NativeContext*>(ctx.ctx.get());
		if (!c) throw std::runtime_error("tcnn::cpp: context was not created by this engine's forward()");
		return c->h;
	}
	tcnn_module* m_h;
};
}  // namespace detail

// cpp_api.h:114-116
inline Module* create_network_with_input_encoding(uint32_t n_input_dims, uint32_t n_output_dims, const json& encoding,
                                                  const json& network) {
	return new detail::NativeModule(
	    tcnn_create_network_with_input_encoding(n_input_dims, n_output_dims, encoding.dump().c_str(), network.dump().c_str()));
}
inline Module* create_network(uint32_t n_input_dims, uint32_t n_output_dims, const json& network) {
	return new detail::NativeModule(tcnn_create_network(n_input_dims, n_output_dims, network.dump().c_str()));
}
inline Module* create_encoding(uint32_t n_input_dims, const json& encoding, Precision requested_precision) {
	return new detail::NativeModule(tcnn_create_encoding(
	    n_input_dims, encoding.dump().c_str(), requested_precision == Precision::Fp16 ? TCNN_PRECISION_FP16 : TCNN_PRECISION_FP32));
}

}}  // namespace tcnn::cpp
