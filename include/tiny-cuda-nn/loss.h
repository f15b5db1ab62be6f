// tiny-cuda-nn/loss.h -- Loss<T> / create_loss<T> (reference include/tiny-cuda-nn/loss.h,
// src/loss.cu) for the MI355X engine. The loss is evaluated inside the engine's training step
// (fused into the MLP kernel); this object carries its configuration into the Trainer.
// Implemented losses: RelativeL2 (losses/relative_l2.h:40-118), L2 (losses/l2.h:40-76).
#pragma once

#include <algorithm>
#include <cctype>

#include "common.h"

namespace tcnn {

namespace detail {
inline bool equals_case_insensitive(const std::string& a, const std::string& b) {
	if (a.size() != b.size()) return false;
	for (size_t i = 0; i < a.size(); ++i)
		if (std::tolower((unsigned char)a[i]) != std::tolower((unsigned char)b[i])) return false;
	return true;
}
}  // namespace detail

template <typename T>
class Loss {
public:
	// (json members are initialised with parentheses: braces would wrap the value in an array)
	explicit Loss(json config) : m_config(std::move(config)) {}
	virtual ~Loss() {}
	void update_hyperparams(const json& params) {
		for (auto it = params.begin(); it != params.end(); ++it) m_config[it.key()] = it.value();
	}
	json hyperparams() const { return m_config; }
	const json& config() const { return m_config; }

private:
	json m_config;
};

// loss.cu: create_loss<T>(json) -- unknown otypes throw as the reference's factory does
template <typename T>
Loss<T>* create_loss(const json& loss) {
	const std::string otype = loss.value("otype", std::string{"RelativeL2"});
	if (!detail::equals_case_insensitive(otype, "RelativeL2") && !detail::equals_case_insensitive(otype, "L2"))
		throw std::runtime_error{"Loss: type '" + otype + "' is not implemented by the MI355X engine (RelativeL2, L2)"};
	json c = loss;
	c["otype"] = otype;
	return new Loss<T>(c);
}

}  // namespace tcnn
