// tiny-cuda-nn/network.h -- Network<T, PARAMS_T> and create_network<T>(json) (reference
// include/tiny-cuda-nn/network.h:44-64, src/network.cu:48-138) for the MI355X engine: the network
// alone, its inputs of type T ([n_input_dims x n]; a Network<__half> takes fp16 inputs). The engine
// runs it as a network behind an Identity encoding of its n_input_dims inputs (cpp_api's
// create_network, tcnn_create_network); a Trainer trains it like any DifferentiableObject.
#pragma once

#include "object.h"

namespace tcnn {

template <typename T, typename PARAMS_T = T>
class Network : public DifferentiableObject<T, PARAMS_T, PARAMS_T> {
public:
	Network(uint32_t n_input_dims, uint32_t n_output_dims, const json& network)
	    : m_n_input_dims{n_input_dims}, m_n_output_dims{n_output_dims}, m_network(network) {
		m_module = detail::check_handle(tcnn_create_network(n_input_dims, n_output_dims, network.dump().c_str()));
	}
	~Network() override { tcnn_module_destroy(m_module); }
	Network(const Network&) = delete;
	Network& operator=(const Network&) = delete;

	uint32_t input_width() const override { return m_n_input_dims; }
	uint32_t output_width() const override { return m_n_output_dims; }
	uint32_t padded_output_width() const override { return tcnn_module_n_output_dims(m_module); }
	size_t n_params() const override { return (size_t)tcnn_module_n_params(m_module); }
	json hyperparams() const override { return json::parse(tcnn_module_hyperparams(m_module)); }
	std::string name() const override { return tcnn_module_name(m_module); }
	json engine_encoding() const override {
		json e = json::object();
		e["otype"] = "Identity";
		return e;
	}
	json engine_network() const override { return m_network; }
	// network.h:54-56 (FullyFusedMLP / CutlassMLP: every hidden layer is n_neurons wide)
	uint32_t width(uint32_t layer) const {
		(void)layer;
		return m_network.value("n_neurons", 128u);
	}
	uint32_t num_forward_activations() const { return m_network.value("n_hidden_layers", 2u); }

private:
	uint32_t m_n_input_dims, m_n_output_dims;
	json m_network;
	tcnn_module* m_module = nullptr;
};

// network.h:60-64: the widths come from the configuration's n_input_dims / n_output_dims
template <typename T>
Network<T, T>* create_network(const json& network) {
	if (!network.count("n_input_dims") || !network.count("n_output_dims"))
		throw std::runtime_error{"create_network: the configuration must give n_input_dims and n_output_dims"};
	return new Network<T, T>(network["n_input_dims"].get<uint32_t>(), network["n_output_dims"].get<uint32_t>(), network);
}

}  // namespace tcnn
