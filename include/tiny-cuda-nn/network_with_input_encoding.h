// tiny-cuda-nn/network_with_input_encoding.h -- NetworkWithInputEncoding<T> (reference
// include/tiny-cuda-nn/network_with_input_encoding.h:41-190, object.h:147-179) for the MI355X engine.
//
// The object carries the encoding + network configuration and reports the model's sizes; its
// parameters live in the Trainer that trains it (the reference's Trainer likewise owns the parameter
// buffers and points the model at them, trainer.h:322-336), so inference() runs on the parameters of
// the attached trainer. Inference before any Trainer owns the network throws, where the reference
// would read unset parameters.
#pragma once

#include "object.h"

namespace tcnn {

template <typename T>
class NetworkWithInputEncoding : public DifferentiableObject<float, T, T> {
public:
	NetworkWithInputEncoding(uint32_t n_dims_to_encode, uint32_t n_output_dims, const json& encoding, const json& network)
	    : m_n_input_dims{n_dims_to_encode}, m_n_output_dims{n_output_dims}, m_encoding(encoding), m_network(network) {
		m_module = detail::check_handle(
		    tcnn_create_network_with_input_encoding(n_dims_to_encode, n_output_dims, encoding.dump().c_str(), network.dump().c_str()));
	}
	~NetworkWithInputEncoding() override { tcnn_module_destroy(m_module); }
	NetworkWithInputEncoding(const NetworkWithInputEncoding&) = delete;
	NetworkWithInputEncoding& operator=(const NetworkWithInputEncoding&) = delete;

	uint32_t input_width() const override { return m_n_input_dims; }
	uint32_t output_width() const override { return m_n_output_dims; }
	uint32_t padded_output_width() const override { return tcnn_module_n_output_dims(m_module); }
	size_t n_params() const override { return (size_t)tcnn_module_n_params(m_module); }
	json hyperparams() const override { return json::parse(tcnn_module_hyperparams(m_module)); }
	std::string name() const override { return tcnn_module_name(m_module); }
	json engine_encoding() const override { return m_encoding; }
	json engine_network() const override { return m_network; }
	const json& encoding_config() const { return m_encoding; }
	const json& network_config() const { return m_network; }

private:
	uint32_t m_n_input_dims, m_n_output_dims;
	json m_encoding, m_network;
	tcnn_module* m_module = nullptr;
};

}  // namespace tcnn
