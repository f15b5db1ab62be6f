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
	Encoding(uint32_t n_dims_to_encode, const json& encoding) : m_n_dims{n_dims_to_encode}, m_encoding(encoding) {
		m_module = detail::check_handle(tcnn_create_encoding(n_dims_to_encode, encoding.dump().c_str(), TCNN_PRECISION_FP16));
	}
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

private:
	uint32_t m_n_dims;
	json m_encoding;
	tcnn_module* m_module = nullptr;
};

// encoding.h:76
template <typename T>
Encoding<T>* create_encoding(uint32_t n_dims_to_encode, const json& params, uint32_t alignment = 8) {
	(void)alignment;  // the engine pads encodings to its own alignment (padded_output_width)
	return new Encoding<T>(n_dims_to_encode, params);
}

}  // namespace tcnn
