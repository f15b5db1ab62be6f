// tiny-cuda-nn/encoding.h -- Encoding<T> and create_encoding<T>(n_dims, json) (reference
// include/tiny-cuda-nn/encoding.h:40-84, src/encoding.cu) for the MI355X engine: a standalone
// encoding (HashGrid / Grid / DenseGrid / OneBlob / Identity), output [padded_output_width() x n].
// Its forward, backward and input gradients run through the runtime Module (tcnn_create_encoding;
// tcnn::cpp::Module in cpp_api.h). The Trainer of this engine trains a network behind an encoding:
// a Trainer constructed over an Encoding alone refuses it (engine_network() is null) rather than
// training something else.
#pragma once

#include "object.h"

namespace tcnn {

template <typename T>
class Encoding : public DifferentiableObject<float, T, T> {
public:
	Encoding(uint32_t n_dims_to_encode, const json& encoding, uint32_t seed = 1337) : m_n_dims{n_dims_to_encode}, m_encoding(encoding) {
		m_module = detail::check_handle(tcnn_create_encoding(n_dims_to_encode, encoding.dump().c_str(), TCNN_PRECISION_FP16));
		// its own parameters (the grid table; none for OneBlob / Identity), initialised as the
		// reference's encodings initialise theirs (grid.h: uniform in +-1e-4), stored fp16
		const size_t n = n_params();
		if (n) {
			GPUMemory<float> p32(n);
			detail::check_rc(tcnn_module_initialize_params(m_module, seed, p32.data(), 1.0f));
			m_params.resize(n);
			hipLaunchKernelGGL(detail::narrow_from_float<__half>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, nullptr, (uint32_t)n, p32.data(),
			                   m_params.data());
			HIP_CHECK_THROW(hipDeviceSynchronize());
		}
	}
	// the parameters inference runs on (fp16, n_params(); the module's precision)
	__half* params() const { return m_params.data(); }
	~Encoding() override { tcnn_module_destroy(m_module); }
	Encoding(const Encoding&) = delete;
	Encoding& operator=(const Encoding&) = delete;

	uint32_t input_width() const override { return m_n_dims; }
	uint32_t output_width() const override { return tcnn_module_n_output_dims(m_module); }
	uint32_t padded_output_width() const override { return tcnn_module_n_output_dims(m_module); }
	size_t n_params() const override { return (size_t)tcnn_module_n_params(m_module); }
	json hyperparams() const override { return json::parse(tcnn_module_hyperparams(m_module)); }
	std::string name() const override { return tcnn_module_name(m_module); }
	json engine_encoding() const override { return m_encoding; }
	json engine_network() const override { return json(); }  // no network: not trainable by this engine's Trainer
	tcnn_module* module() const { return m_module; }

protected:
	// object.h inference without a Trainer: the module's forward on this encoding's own parameters,
	// fp16 output widened into the fp32 matrix
	bool inference_standalone(hipStream_t stream, const GPUMatrixDynamic<float>& input, GPUMatrixDynamic<float>& output) override {
		const uint32_t n = input.n(), w = padded_output_width();
		m_out16.enlarge((size_t)n * w);
		detail::check_rc(tcnn_module_inference(m_module, stream, n, input.data(), m_out16.data(), m_params.data()));
		const uint32_t ne = n * w;
		if (ne) hipLaunchKernelGGL(detail::widen_to_float<__half>, dim3((ne + 255) / 256), dim3(256), 0, stream, ne, m_out16.data(), output.data());
		return true;
	}

private:
	uint32_t m_n_dims;
	json m_encoding;
	tcnn_module* m_module = nullptr;
	GPUMemory<__half> m_params;
	GPUMemory<__half> m_out16;
};

// encoding.h:76
template <typename T>
Encoding<T>* create_encoding(uint32_t n_dims_to_encode, const json& params, uint32_t alignment = 8) {
	(void)alignment;  // the engine pads encodings to its own alignment (padded_output_width)
	return new Encoding<T>(n_dims_to_encode, params);
}

}  // namespace tcnn
