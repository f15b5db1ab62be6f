// tiny-cuda-nn/trainer.h -- Trainer<T, PARAMS_T, COMPUTE_T> (reference
// include/tiny-cuda-nn/trainer.h:47-361) for the MI355X engine.
//
// The engine runs forward, loss, backward and (optionally) the optimizer of one training step as
// three launches on the caller's stream (neuralbtf-tiny-cuda-nn_amd/csrc/runtime.cpp,
// TrainerHost::training_step_overlapped), so training_step() is one C-ABI call. The ForwardContext it
// returns holds a copy of that step's loss sum on the device; loss(ctx) reads it for any live context
// (trainer.h:205-211 reduces the context's loss values). With any of the reference's options (data_pdf, external dL/dy, dL/dinput,
// Accumulate gradients) training_step runs as the reference's does: forward() (network output +
// loss, or the caller's dL/dy) then backward() (tcnn_trainer_forward / _backward), then the optimizer;
// loss(ctx) then reads the context's own loss. Output perturbation (perturbation_sigma > 0) runs the
// same way, with the reference's logistic noise on the output the loss sees.
#pragma once

#include <memory>
#include <random>
#include <vector>

#include "encoding.h"
#include "network.h"
#include "network_with_input_encoding.h"
#include "optimizer.h"
#include "random.h"

namespace tcnn {

template <typename T, typename PARAMS_T, typename COMPUTE_T = T>
class Trainer {
public:
	// trainer.h:50: any DifferentiableObject -- NetworkWithInputEncoding, Network (create_network; inputs
	// of type T, fp16 ones widened for the engine), not an Encoding alone (refused below)
	using Model = DifferentiableObject<T, PARAMS_T, COMPUTE_T>;

	// trainer.h:50-57: the trainer owns the parameters (seeded pcg32{seed_seq{seed}[0]})
	Trainer(std::shared_ptr<Model> model, std::shared_ptr<Optimizer<PARAMS_T>> optimizer, std::shared_ptr<Loss<COMPUTE_T>> loss,
	        uint32_t seed = 1337, float perturbation_sigma = 0)
	    : m_model{std::move(model)}, m_optimizer{std::move(optimizer)}, m_loss{std::move(loss)}, m_seed{seed},
	      m_perturbation_sigma{perturbation_sigma} {
		static_assert(std::is_same<T, float>::value || std::is_same<T, __half>::value, "Trainer: inputs are fp32 or fp16");
		if (m_model->engine_network().is_null())
			throw std::runtime_error{"Trainer: " + m_model->name() + " has no network; this engine trains a network behind an encoding "
			                         "(NetworkWithInputEncoding, or Network for the network alone)"};
		// (keyed assignment: brace-initialising with json values would wrap them in arrays)
		json cfg = json::object();
		cfg["loss"] = m_loss->config();
		cfg["optimizer"] = m_optimizer->config();
		cfg["encoding"] = m_model->engine_encoding();
		cfg["network"] = m_model->engine_network();
		m_h = detail::check_handle(tcnn_trainer_create(m_model->input_width(), m_model->output_width(), cfg.dump().c_str(), seed));
		m_model->attach(m_h);
		m_optimizer->attach(m_h);
		reset_rng();
	}
	virtual ~Trainer() {
		if (m_model->trainer_handle() == m_h) m_model->attach(nullptr);
		m_optimizer->attach(nullptr);
		tcnn_trainer_destroy(m_h);
	}
	Trainer(const Trainer&) = delete;
	Trainer& operator=(const Trainer&) = delete;

	// trainer.h:89-95. A context made by forward() (or an optioned training_step) owns the engine's
	// context: output and dL_doutput are views of its fp16 [padded_output_width x batch] buffers.
	// Device slots holding the loss of each live fused-step context: the fused step keeps one loss sum,
	// so training_step copies it (stream-ordered, 4 bytes) into the context's own slot and loss(ctx)
	// reads that -- any live context, as the reference's loss(ctx) reduces the context's own values.
	struct LossSlots {
		std::vector<GPUMemory<float>> blocks;
		std::vector<float*> free_list;
		static constexpr size_t BLOCK = 1024;
		float* take() {
			if (free_list.empty()) {
				blocks.emplace_back(BLOCK);
				for (size_t k = 0; k < BLOCK; ++k) free_list.push_back(blocks.back().data() + (BLOCK - 1 - k));
			}
			float* p = free_list.back();
			free_list.pop_back();
			return p;
		}
	};
	struct ForwardContext : public Context {
		const Trainer* owner = nullptr;
		uint64_t step = 0;
		tcnn_trainer_context* h = nullptr;
		GPUMatrix<COMPUTE_T> output, dL_doutput;
		std::shared_ptr<LossSlots> slots;  // a fused step's loss slot (returned on destruction)
		float* loss_slot = nullptr;
		GPUMemory<float> input_f32;  // Trainer<__half, ...>: the widened input the engine read (for backward)
		ForwardContext() = default;
		ForwardContext(const ForwardContext&) = delete;
		ForwardContext& operator=(const ForwardContext&) = delete;
		~ForwardContext() {
			tcnn_trainer_context_destroy(h);
			if (slots && loss_slot) slots->free_list.push_back(loss_slot);
		}
	};

	uint32_t padded_output_width() const { return tcnn_trainer_padded_output_width(m_h); }

	// trainer.h:97-144: network output + loss (or the caller's external dL/dy, loss-scaled)
	std::unique_ptr<ForwardContext> forward(hipStream_t stream, const float loss_scale, const GPUMatrixDynamic<T>& input,
	                                        const GPUMatrixDynamic<float>& target, const GPUMatrixDynamic<float>* data_pdf = nullptr,
	                                        bool use_inference_params = false, bool prepare_input_gradients = false,
	                                        const GPUMatrixDynamic<COMPUTE_T>* external_dL_dy = nullptr) {
		(void)loss_scale;  // the engine's default_loss_scale<__half>() (common.h:232)
		(void)use_inference_params;
		const uint32_t n = input.n();
		CHECK_THROW(input.m() == m_model->input_width());
		CHECK_THROW(input.layout() == CM && input.is_contiguous());
		if (external_dL_dy) {
			CHECK_THROW(external_dL_dy->m() == padded_output_width());
			CHECK_THROW(external_dL_dy->n() == n);
		} else {
			CHECK_THROW(target.m() == m_model->output_width());
			CHECK_THROW(target.n() == n);
		}
		if (data_pdf) CHECK_THROW(data_pdf->m() == m_model->output_width() && data_pdf->n() == n);
		auto ctx = std::make_unique<ForwardContext>();
		ctx->owner = this;
		ctx->step = ++m_n_steps;
		const float* in = detail::engine_input(stream, input, ctx->input_f32);
		if (m_perturbation_sigma > 0) {
			// trainer.h:114-123: logistic noise (m_rng) drawn on every forward -- with an external dL/dy too,
			// so the generator advances as the reference's -- and added to the output; the loss and dL/dy see
			// the perturbed output, the context's output stays unperturbed
			const size_t n_el = (size_t)padded_output_width() * n;
			m_perturbation.enlarge(n_el);
			generate_random_logistic(stream, m_rng, n_el, m_perturbation.data(), 0.0f, m_perturbation_sigma);
		}
		if (m_perturbation_sigma > 0 && !external_dL_dy) {
			ctx->h = tcnn_trainer_forward_perturbed(m_h, stream, n, in, target.data(), data_pdf ? data_pdf->data() : nullptr,
			                                        m_perturbation.data(), prepare_input_gradients ? 1 : 0);
		} else {
			ctx->h = tcnn_trainer_forward(m_h, stream, n, in, external_dL_dy ? nullptr : target.data(),
			                              data_pdf ? data_pdf->data() : nullptr, external_dL_dy ? external_dL_dy->data() : nullptr,
			                              prepare_input_gradients ? 1 : 0);
		}
		if (!ctx->h) throw std::runtime_error{tcnn_last_error()};
		const uint32_t w = padded_output_width();
		ctx->output = GPUMatrix<COMPUTE_T>{(COMPUTE_T*)tcnn_trainer_context_output(ctx->h), w, n};
		ctx->dL_doutput = GPUMatrix<COMPUTE_T>{(COMPUTE_T*)tcnn_trainer_context_doutput(ctx->h), w, n};
		return ctx;
	}
	std::unique_ptr<ForwardContext> forward(const float loss_scale, const GPUMatrixDynamic<T>& input, const GPUMatrixDynamic<float>& target,
	                                        const GPUMatrixDynamic<float>* data_pdf = nullptr, bool use_inference_params = false,
	                                        bool prepare_input_gradients = false,
	                                        const GPUMatrixDynamic<COMPUTE_T>* external_dL_dy = nullptr) {
		return forward(nullptr, loss_scale, input, target, data_pdf, use_inference_params, prepare_input_gradients, external_dL_dy);
	}

	// trainer.h:146-153: parameter gradients (Overwrite or Accumulate) and optionally dL/dinput
	void backward(hipStream_t stream, const ForwardContext& ctx, const GPUMatrixDynamic<T>& input, GPUMatrixDynamic<T>* dL_dinput = nullptr,
	              bool use_inference_params = false, GradientMode param_gradients_mode = GradientMode::Overwrite) {
		(void)use_inference_params;
		if (!ctx.h || ctx.owner != this) throw std::runtime_error{"Trainer::backward: the context was not made by this trainer's forward()"};
		if (dL_dinput) CHECK_THROW(dL_dinput->m() == m_model->input_width() && dL_dinput->n() == input.n() && dL_dinput->layout() == CM);
		const int mode = param_gradients_mode == GradientMode::Overwrite ? 0 : param_gradients_mode == GradientMode::Accumulate ? 1 : 2;
		if constexpr (std::is_same<T, float>::value) {
			detail::check_rc(tcnn_trainer_backward(m_h, stream, ctx.h, input.n(), input.data(), dL_dinput ? dL_dinput->data() : nullptr, mode));
		} else {
			// the engine's fp32 input of this context's forward; fp32 dL/dinput narrowed to T
			CHECK_THROW(ctx.input_f32.size() >= input.n_elements());
			GPUMemory<float> din32(dL_dinput ? dL_dinput->n_elements() : 0);
			detail::check_rc(tcnn_trainer_backward(m_h, stream, ctx.h, input.n(), ctx.input_f32.data(), dL_dinput ? din32.data() : nullptr, mode));
			if (dL_dinput) {
				const uint32_t ne = (uint32_t)dL_dinput->n_elements();
				hipLaunchKernelGGL(detail::narrow_from_float<T>, dim3((ne + 255) / 256), dim3(256), 0, stream, ne, din32.data(), dL_dinput->data());
				HIP_CHECK_THROW(hipStreamSynchronize(stream));  // din32 is freed on return
			}
		}
	}
	void backward(const ForwardContext& ctx, const GPUMatrixDynamic<T>& input, GPUMatrixDynamic<T>* dL_dinput = nullptr,
	              bool use_inference_params = false, GradientMode param_gradients_mode = GradientMode::Overwrite) {
		backward(nullptr, ctx, input, dL_dinput, use_inference_params, param_gradients_mode);
	}

	// trainer.h:68-87
	void initialize_params() {
		// from m_rng, which keeps advancing (the reference re-initialises from its live generator, not
		// from the seed): a second call draws new values, as the reference's does
		uint64_t state = m_rng.state;
		detail::check_rc(tcnn_trainer_initialize_params_rng(m_h, &state, m_rng.inc));
		m_rng.state = state;  // the generator as the engine left it (however many values it drew)
		++m_n_steps;  // contexts of earlier steps no longer describe the parameters
	}

	// trainer.h:163-203
	std::unique_ptr<ForwardContext> training_step(hipStream_t stream, const GPUMatrixDynamic<T>& input, const GPUMatrixDynamic<float>& target,
	                                              const GPUMatrixDynamic<float>* data_pdf = nullptr, bool run_optimizer = true,
	                                              GPUMatrixDynamic<T>* dL_dinput = nullptr, bool use_inference_params = false,
	                                              GradientMode param_gradients_mode = GradientMode::Overwrite,
	                                              const GPUMatrixDynamic<COMPUTE_T>* external_dL_dy = nullptr) {
		(void)use_inference_params;
		CHECK_THROW(input.m() == m_model->input_width());
		CHECK_THROW(input.n() % BATCH_SIZE_GRANULARITY == 0);
		CHECK_THROW(input.layout() == CM && input.is_contiguous());
		if (data_pdf || dL_dinput || external_dL_dy || param_gradients_mode != GradientMode::Overwrite || m_perturbation_sigma > 0) {
			// trainer.h:163-203 as written: forward, backward, optimizer
			auto ctx = forward(stream, default_loss_scale<PARAMS_T>(), input, target, data_pdf, use_inference_params, dL_dinput != nullptr,
			                   external_dL_dy);
			backward(stream, *ctx, input, dL_dinput, use_inference_params, param_gradients_mode);
			if (run_optimizer) optimizer_step(stream, default_loss_scale<PARAMS_T>());
			return ctx;
		}
		CHECK_THROW(target.m() == m_model->output_width());
		CHECK_THROW(input.n() == target.n());
		CHECK_THROW(target.layout() == CM && target.is_contiguous());
		const float* in = detail::engine_input(stream, input, m_input_scratch);
		detail::check_rc(tcnn_trainer_training_step(m_h, stream, input.n(), in, target.data(), run_optimizer ? 1 : 0));
		auto ctx = std::make_unique<ForwardContext>();
		ctx->owner = this;
		ctx->step = ++m_n_steps;
		ctx->slots = m_loss_slots;
		ctx->loss_slot = m_loss_slots->take();
		HIP_CHECK_THROW(hipMemcpyAsync(ctx->loss_slot, tcnn_trainer_loss_device(m_h), sizeof(float), hipMemcpyDeviceToDevice, stream));
		return ctx;
	}
	std::unique_ptr<ForwardContext> training_step(const GPUMatrixDynamic<T>& input, const GPUMatrixDynamic<float>& target,
	                                              const GPUMatrixDynamic<float>* data_pdf = nullptr, bool run_optimizer = true,
	                                              GPUMatrixDynamic<T>* dL_dinput = nullptr, bool use_inference_params = false,
	                                              GradientMode param_gradients_mode = GradientMode::Overwrite,
	                                              const GPUMatrixDynamic<COMPUTE_T>* external_dL_dy = nullptr) {
		return training_step(nullptr, input, target, data_pdf, run_optimizer, dL_dinput, use_inference_params, param_gradients_mode,
		                     external_dL_dy);
	}

	// trainer.h:205-211: synchronises `stream`
	float loss(hipStream_t stream, const ForwardContext& ctx) const {
		if (ctx.h && ctx.owner == this) {  // a forward() context carries its own loss values
			const float v = tcnn_trainer_context_loss(m_h, stream, ctx.h);
			if (v < 0.0f) throw std::runtime_error{tcnn_last_error()};
			return v;
		}
		if (ctx.owner != this || !ctx.loss_slot) throw std::runtime_error{"Trainer::loss: the context was not made by this trainer"};
		float v = 0.0f;
		HIP_CHECK_THROW(hipMemcpyAsync(&v, ctx.loss_slot, sizeof(float), hipMemcpyDeviceToHost, stream));
		HIP_CHECK_THROW(hipStreamSynchronize(stream));
		return v;
	}
	float loss(const ForwardContext& ctx) const { return loss(nullptr, ctx); }

	// trainer.h:155-161 (the loss scale is the engine's default_loss_scale<PARAMS_T>())
	void optimizer_step(hipStream_t stream, float loss_scale) {
		(void)loss_scale;
		detail::check_rc(tcnn_trainer_optimizer_step(m_h, stream));
	}
	void optimizer_step(float loss_scale) { optimizer_step(nullptr, loss_scale); }

	// trainer.h:213-224
	void update_hyperparams(const json& params) {
		if (params.count("optimizer")) m_optimizer->update_hyperparams(params["optimizer"]);
		if (params.count("loss")) {
			// the engine's loss is fixed at construction: it refuses an otype change instead of
			// silently training on with the old loss (tcnn_trainer_update_hyperparams)
			json l = json::object();
			l["loss"] = params["loss"];
			detail::check_rc(tcnn_trainer_update_hyperparams(m_h, l.dump().c_str()));
			m_loss->update_hyperparams(params["loss"]);
		}
	}
	json hyperparams() const { return json::parse(tcnn_trainer_hyperparams(m_h)); }

	// parameter buffers (trainer.h:226-240, 322-336): device pointers owned by the trainer
	float* params_full_precision() const { return tcnn_trainer_params_fp32(m_h); }
	PARAMS_T* params() const { return (PARAMS_T*)tcnn_trainer_params(m_h); }
	PARAMS_T* params_inference() const { return params(); }
	PARAMS_T* param_gradients() const { return (PARAMS_T*)tcnn_trainer_param_gradients(m_h); }
	size_t n_params() const { return (size_t)tcnn_trainer_n_params(m_h); }

	// trainer.h:242-273
	void set_params_full_precision(const float* params, size_t n_params, bool device_ptr = false) {
		if (n_params != this->n_params()) throw std::runtime_error{"Can't set fp params because buffer has the wrong size."};
		std::vector<float> host;
		if (device_ptr) {
			host.resize(n_params);
			HIP_CHECK_THROW(hipMemcpy(host.data(), params, n_params * sizeof(float), hipMemcpyDeviceToHost));
			params = host.data();
		}
		detail::check_rc(tcnn_trainer_set_params_full_precision(m_h, params, n_params));
	}
	void set_params(const PARAMS_T* params, size_t n_params, bool device_ptr = false) {
		if (n_params != this->n_params()) throw std::runtime_error{"Can't set params because buffer has the wrong size."};
		std::vector<PARAMS_T> h(n_params);
		if (device_ptr) HIP_CHECK_THROW(hipMemcpy(h.data(), params, n_params * sizeof(PARAMS_T), hipMemcpyDeviceToHost));
		else std::copy(params, params + n_params, h.begin());
		std::vector<float> f(n_params);
		for (size_t i = 0; i < n_params; ++i) f[i] = (float)h[i];
		detail::check_rc(tcnn_trainer_set_params_full_precision(m_h, f.data(), n_params));
	}

	// trainer.h:275-315: json::to_msgpack(serialize(optimizer)) bytes and back (nlohmann 3.1.1, the
	// json library of this toolchain, has no binary values, so the msgpack image is the interface)
	std::vector<uint8_t> serialize_msgpack(bool serialize_optimizer = false) {
		uint64_t n = 0;
		detail::check_rc(tcnn_trainer_serialize(m_h, serialize_optimizer ? 1 : 0, nullptr, 0, &n));
		std::vector<uint8_t> out(n);
		detail::check_rc(tcnn_trainer_serialize(m_h, serialize_optimizer ? 1 : 0, out.data(), n, &n));
		out.resize(n);
		return out;
	}
	void deserialize_msgpack(const std::vector<uint8_t>& data) {
		detail::check_rc(tcnn_trainer_deserialize(m_h, data.data(), data.size()));
	}
	// trainer.h:275-315 with the reference's signatures: json::to_msgpack(trainer->serialize(true)) and
	// trainer->deserialize(json::from_msgpack(...)) read the same. This json library (nlohmann 3.1.1)
	// has no binary type, so the binaries travel as nlohmann's binary-as-JSON object
	// {"bytes": [u8...], "subtype": null}; deserialize accepts that form and the msgpack image alike.
	json serialize(bool serialize_optimizer = false) {
		uint64_t n = 0;
		detail::check_rc(tcnn_trainer_serialize_json(m_h, serialize_optimizer ? 1 : 0, nullptr, 0, &n));
		std::string text(n, '\0');
		detail::check_rc(tcnn_trainer_serialize_json(m_h, serialize_optimizer ? 1 : 0, &text[0], n, &n));
		text.resize(n ? n - 1 : 0);
		return json::parse(text);
	}
	void deserialize(const json& data) {
		const std::string text = data.dump();
		detail::check_rc(tcnn_trainer_deserialize(m_h, text.data(), text.size()));
	}

	std::shared_ptr<Model> model() const { return m_model; }
	std::shared_ptr<Optimizer<PARAMS_T>> optimizer() const { return m_optimizer; }
	std::shared_ptr<Loss<COMPUTE_T>> loss_object() const { return m_loss; }
	// which of the engine's paths trains this model ("fused" / "layered")
	std::string engine() const { return tcnn_trainer_engine(m_h); }
	tcnn_trainer* handle() const { return m_h; }
	float perturbation_sigma() const { return m_perturbation_sigma; }

private:
	// trainer.h:52-55, 68-87: the trainer's pcg32{seed_seq{seed}[0]} after the parameter initialisation
	// drew its n_params uniforms (generate_random_uniform advances by n_elements, random.h:64) -- the
	// engine initialises from the same seed, so this is the state the reference's m_rng has when the
	// first perturbation is drawn
	void reset_rng() {
		std::seed_seq seq{m_seed};
		std::vector<uint32_t> seeds(2);
		seq.generate(std::begin(seeds), std::end(seeds));
		m_rng = default_rng_t{seeds.front()};
		m_rng.advance((int64_t)n_params());
	}

	std::shared_ptr<Model> m_model;
	std::shared_ptr<Optimizer<PARAMS_T>> m_optimizer;
	std::shared_ptr<Loss<COMPUTE_T>> m_loss;
	uint32_t m_seed;
	float m_perturbation_sigma;
	default_rng_t m_rng;
	GPUMemory<float> m_perturbation;
	tcnn_trainer* m_h = nullptr;
	uint64_t m_n_steps = 0;
	GPUMemory<float> m_input_scratch;  // Trainer<__half, ...>: the widened batch of training_step
	std::shared_ptr<LossSlots> m_loss_slots = std::make_shared<LossSlots>();
};

}  // namespace tcnn
