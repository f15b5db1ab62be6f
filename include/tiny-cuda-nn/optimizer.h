// tiny-cuda-nn/optimizer.h -- Optimizer<T> / create_optimizer<T> (reference
// include/tiny-cuda-nn/optimizer.h, src/optimizer.cu) for the MI355X engine. Adam
// (optimizers/adam.h:47-327) runs inside the engine's training step; this object carries its
// configuration into the Trainer and forwards later hyper-parameter changes to it.
#pragma once

#include "loss.h"

namespace tcnn {

template <typename T>
class Optimizer {
public:
	explicit Optimizer(json config) : m_config(std::move(config)) {}
	virtual ~Optimizer() {}

	// adam.h:235-283 / 200-210
	void update_hyperparams(const json& params) {
		for (auto it = params.begin(); it != params.end(); ++it) m_config[it.key()] = it.value();
		if (m_trainer) {
			json p = json::object();
			p["optimizer"] = params;
			detail::check_rc(tcnn_trainer_update_hyperparams(m_trainer, p.dump().c_str()));
		}
	}
	json hyperparams() const {
		if (m_trainer) return json::parse(tcnn_trainer_hyperparams(m_trainer))["optimizer"];
		return m_config;
	}
	float learning_rate() const { return hyperparams().value("learning_rate", 1e-3f); }
	void set_learning_rate(float lr) { update_hyperparams({{"learning_rate", lr}}); }
	uint32_t step() const { return m_trainer ? tcnn_trainer_optimizer_step_count(m_trainer) : 0u; }
	const json& config() const { return m_config; }

	// set by the Trainer that runs this optimizer
	void attach(tcnn_trainer* t) { m_trainer = t; }

private:
	json m_config;
	tcnn_trainer* m_trainer = nullptr;
};

template <typename T>
Optimizer<T>* create_optimizer(const json& optimizer) {
	const std::string otype = optimizer.value("otype", std::string{"Adam"});
	if (!detail::equals_case_insensitive(otype, "Adam"))
		throw std::runtime_error{"Optimizer: type '" + otype + "' is not implemented by the MI355X engine (Adam)"};
	json c = optimizer;
	c["otype"] = otype;
	return new Optimizer<T>(c);
}

}  // namespace tcnn
