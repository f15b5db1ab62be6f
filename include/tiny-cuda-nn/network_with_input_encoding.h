// tiny-cuda-nn/network_with_input_encoding.h -- NetworkWithInputEncoding<T> (reference
// include/tiny-cuda-nn/network_with_input_encoding.h:41-190, object.h:147-179) for the MI355X engine.
//
// The object carries the encoding + network configuration and reports the model's sizes; its
// parameters live in the Trainer that trains it (the reference's Trainer likewise owns the parameter
// buffers and points the model at them, trainer.h:322-336), so inference() runs on the parameters of
// the attached trainer. Inference before any Trainer owns the network throws, where the reference
// would read unset parameters.
#pragma once

#include "gpu_matrix.h"

namespace tcnn {

template <typename T>
class NetworkWithInputEncoding {
public:
	NetworkWithInputEncoding(uint32_t n_dims_to_encode, uint32_t n_output_dims, const json& encoding, const json& network)
	    : m_n_input_dims{n_dims_to_encode}, m_n_output_dims{n_output_dims}, m_encoding(encoding), m_network(network) {
		m_module = detail::check_handle(
		    tcnn_create_network_with_input_encoding(n_dims_to_encode, n_output_dims, encoding.dump().c_str(), network.dump().c_str()));
	}
	virtual ~NetworkWithInputEncoding() { tcnn_module_destroy(m_module); }
	NetworkWithInputEncoding(const NetworkWithInputEncoding&) = delete;
	NetworkWithInputEncoding& operator=(const NetworkWithInputEncoding&) = delete;

	// object.h:147-176: output fp32 [output_width() x n] from input [input_width() x n], n a multiple of 256
	void inference(hipStream_t stream, const GPUMatrixDynamic<float>& input, GPUMatrixDynamic<float>& output, bool use_inference_params = true) {
		(void)use_inference_params;  // one parameter set: the trainer's fp16 parameters
		CHECK_THROW(input.m() == input_width());
		CHECK_THROW(output.m() == output_width());
		CHECK_THROW(input.n() % BATCH_SIZE_GRANULARITY == 0);
		CHECK_THROW(input.n() == output.n());
		CHECK_THROW(input.layout() == CM && input.is_contiguous() && output.layout() == CM && output.is_contiguous());
		if (!m_trainer) throw std::runtime_error{"NetworkWithInputEncoding::inference: no parameters (the network is not owned by a Trainer)"};
		detail::check_rc(tcnn_trainer_inference(m_trainer, stream, input.n(), input.data(), output.data()));
	}
	void inference(const GPUMatrixDynamic<float>& input, GPUMatrixDynamic<float>& output, bool use_inference_params = true) {
		inference(nullptr, input, output, use_inference_params);
	}

	uint32_t input_width() const { return m_n_input_dims; }
	uint32_t output_width() const { return m_n_output_dims; }
	uint32_t padded_output_width() const { return tcnn_module_n_output_dims(m_module); }
	size_t n_params() const { return (size_t)tcnn_module_n_params(m_module); }
	json hyperparams() const { return json::parse(tcnn_module_hyperparams(m_module)); }
	std::string name() const { return tcnn_module_name(m_module); }
	const json& encoding_config() const { return m_encoding; }
	const json& network_config() const { return m_network; }

	// set by the Trainer that owns this network's parameters
	void attach(tcnn_trainer* t) { m_trainer = t; }
	tcnn_trainer* trainer_handle() const { return m_trainer; }

private:
	uint32_t m_n_input_dims, m_n_output_dims;
	json m_encoding, m_network;
	tcnn_module* m_module = nullptr;
	tcnn_trainer* m_trainer = nullptr;
};

}  // namespace tcnn
