// tiny-cuda-nn/config.h -- create_from_config() / TrainableModel (reference
// include/tiny-cuda-nn/config.h:46-63) for the MI355X engine: loss, optimizer, network and trainer
// from one JSON object {"loss", "optimizer", "encoding", "network"}.
#pragma once

#include "common_device.h"
#include "trainer.h"

namespace tcnn {

struct TrainableModel {
	std::shared_ptr<Loss<network_precision_t>> loss;
	std::shared_ptr<Optimizer<network_precision_t>> optimizer;
	std::shared_ptr<NetworkWithInputEncoding<network_precision_t>> network;
	std::shared_ptr<Trainer<float, network_precision_t, network_precision_t>> trainer;
};

inline TrainableModel create_from_config(uint32_t n_input_dims, uint32_t n_output_dims, json config) {
	std::shared_ptr<Loss<network_precision_t>> loss{create_loss<network_precision_t>(config.value("loss", json::object()))};
	std::shared_ptr<Optimizer<network_precision_t>> optimizer{create_optimizer<network_precision_t>(config.value("optimizer", json::object()))};
	auto network = std::make_shared<NetworkWithInputEncoding<network_precision_t>>(
	    n_input_dims, n_output_dims, config.value("encoding", json::object()), config.value("network", json::object()));
	auto trainer = std::make_shared<Trainer<float, network_precision_t, network_precision_t>>(network, optimizer, loss);
	return {loss, optimizer, network, trainer};
}

}  // namespace tcnn
