// torch_ext.cpp -- the torch autograd node of tinycudann.Module in C++ (r06):
// the reference's `_module_function` / `_module_function_backward` (bindings/torch/tinycudann/
// modules.py:91-192, over bindings.cpp:79-171) as torch::autograd::Function subclasses calling the same
// C-ABI entry points (include/tcnn_mi355x.h) the Python front-end calls through ctypes. One pybind call
// per forward and no Python frame in the backward: the step's host cost was the Python autograd
// plumbing around the engine's calls (profiles/r05_torch_host.json). Host-only code: the device work
// is the engine's. Same arithmetic and null-tensor conventions as the Python path, which stays as the
// fallback (tinycudann.modules uses this module when it has been built).
#include <torch/extension.h>

#include <c10/hip/HIPStream.h>

#include "../../include/tcnn_mi355x.h"

namespace {

void check(int rc) { TORCH_CHECK(rc == 0, "tinycudann (MI355X): ", tcnn_last_error()); }

void* stream_of(const torch::Tensor& t) { return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

torch::ScalarType precision_dtype(int p) { return p == 1 ? torch::kHalf : torch::kFloat; }

void* ptr(const torch::Tensor& t) { return t.defined() ? t.data_ptr() : nullptr; }

// the engine's forward context of one autograd node, destroyed with the node
struct NativeCtx : torch::CustomClassHolder {
	tcnn_context* c = nullptr;
	explicit NativeCtx(tcnn_context* ctx) : c(ctx) {}
	~NativeCtx() override {
		if (c) tcnn_context_destroy(c);
	}
};

tcnn_context* native(const torch::autograd::AutogradContext* ctx) {
	const auto v = ctx->saved_data.at("native");
	return v.isNone() ? nullptr : v.toCustomClass<NativeCtx>()->c;
}

tcnn_module* module_of(const torch::autograd::AutogradContext* ctx) { return (tcnn_module*)ctx->saved_data.at("module").toInt(); }

// reference modules.py:128-170: the first-order backward as a differentiable function (only taken when
// the backward itself is recorded, create_graph=True), whose backward is Module::backward_backward_input
struct ModuleBackward : public torch::autograd::Function<ModuleBackward> {
	static torch::autograd::variable_list forward(torch::autograd::AutogradContext* ctx, int64_t module, c10::IValue native_ctx,
	                                              double loss_scale, torch::Tensor doutput, torch::Tensor input, torch::Tensor params,
	                                              torch::Tensor output) {
		tcnn_module* m = (tcnn_module*)module;
		ctx->saved_data["module"] = module;
		ctx->saved_data["native"] = native_ctx;
		ctx->saved_data["loss_scale"] = loss_scale;
		ctx->save_for_backward({input, params, doutput});
		torch::NoGradGuard ng;
		const int64_t B = input.size(0);
		const torch::Tensor scaled = (doutput * loss_scale).to(precision_dtype(tcnn_module_output_precision(m))).contiguous();
		torch::Tensor gin = input.requires_grad() ? torch::empty_like(input) : torch::Tensor();
		torch::Tensor gpar = params.requires_grad() ? torch::empty({(int64_t)tcnn_module_n_params(m)}, params.options()) : torch::Tensor();
		tcnn_context* c = native_ctx.isNone() ? nullptr : native_ctx.toCustomClass<NativeCtx>()->c;
		check(tcnn_module_backward(m, stream_of(input), c, (uint32_t)B, (float*)ptr(gin), ptr(scaled), ptr(gpar), (const float*)ptr(input),
		                           ptr(output), ptr(params)));
		gin = gin.defined() ? gin / loss_scale : torch::empty({}, input.options());  // null tensors as the reference
		gpar = gpar.defined() ? gpar / loss_scale : torch::empty({}, params.options());
		return {gin, gpar};
	}

	static torch::autograd::variable_list backward(torch::autograd::AutogradContext* ctx, torch::autograd::variable_list grads) {
		const auto saved = ctx->get_saved_variables();
		const torch::Tensor input = saved[0], params = saved[1], doutput_saved = saved[2];
		const torch::Tensor dinput_grad = grads[0];
		torch::autograd::variable_list none(7);
		if (!dinput_grad.defined()) return none;
		tcnn_module* m = module_of(ctx);
		const double ls = ctx->saved_data.at("loss_scale").toDouble();
		torch::Tensor doutput;
		{
			torch::AutoGradMode g(true);
			doutput = doutput_saved * ls;
		}
		torch::NoGradGuard ng;
		const int64_t B = input.size(0);
		const torch::Device dev = input.device();
		const auto odt = precision_dtype(tcnn_module_output_precision(m)), pdt = precision_dtype(tcnn_module_param_precision(m));
		torch::Tensor ddout = doutput_saved.requires_grad()
		                          ? torch::zeros({B, (int64_t)tcnn_module_n_output_dims(m)}, torch::TensorOptions().dtype(odt).device(dev))
		                          : torch::Tensor();
		torch::Tensor dpar = params.requires_grad() ? torch::zeros({(int64_t)tcnn_module_n_params(m)}, torch::TensorOptions().dtype(pdt).device(dev))
		                                            : torch::Tensor();
		torch::Tensor din = input.requires_grad() ? torch::zeros({B, (int64_t)tcnn_module_n_input_dims(m)}, torch::TensorOptions().dtype(torch::kFloat).device(dev))
		                                          : torch::Tensor();
		if (doutput_saved.requires_grad() || params.requires_grad()) {
			const torch::Tensor ddl = dinput_grad.to(torch::kFloat).contiguous();
			const torch::Tensor dout = doutput.detach().to(odt).contiguous();
			check(tcnn_module_backward_backward_input(m, stream_of(input), native(ctx), (uint32_t)B, (const float*)ptr(ddl), (const float*)ptr(input),
			                                          (params.requires_grad() || input.requires_grad()) ? ptr(dout) : nullptr, ptr(dpar),
			                                          ptr(ddout), (float*)ptr(din), ptr(params)));
		}
		if (dpar.defined()) dpar = dpar / ls;
		if (din.defined()) din = din / ls;
		// inputs: module, native_ctx, loss_scale, doutput, input, params, output
		return {torch::Tensor(), torch::Tensor(), torch::Tensor(), ddout, din, dpar, torch::Tensor()};
	}
};

// reference modules.py:91-126 (_module_function)
struct ModuleFunction : public torch::autograd::Function<ModuleFunction> {
	static torch::Tensor forward(torch::autograd::AutogradContext* ctx, int64_t module, torch::Tensor input, torch::Tensor params, double loss_scale) {
		tcnn_module* m = (tcnn_module*)module;
		ctx->set_materialize_grads(false);
		TORCH_CHECK(input.scalar_type() == torch::kFloat && input.is_contiguous() && input.size(1) == (int64_t)tcnn_module_n_input_dims(m),
		            "tinycudann: input must be contiguous fp32 [B, n_input_dims]");
		TORCH_CHECK(params.scalar_type() == precision_dtype(tcnn_module_param_precision(m)) && params.numel() == (int64_t)tcnn_module_n_params(m),
		            "tinycudann: params of the wrong precision or size");
		const int64_t B = input.size(0);
		torch::Tensor out = torch::empty({B, (int64_t)tcnn_module_n_output_dims(m)},
		                                 torch::TensorOptions().dtype(precision_dtype(tcnn_module_output_precision(m))).device(input.device()));
		c10::IValue nctx;  // None: inference (no gradient will be asked for)
		if (!(input.requires_grad() || params.requires_grad())) {
			check(tcnn_module_inference(m, stream_of(input), (uint32_t)B, (const float*)ptr(input), ptr(out), ptr(params)));
		} else {
			tcnn_context* c = tcnn_module_forward(m, stream_of(input), (uint32_t)B, (const float*)ptr(input), ptr(out), ptr(params),
			                                      input.requires_grad() ? 1 : 0);
			TORCH_CHECK(c != nullptr, "tinycudann (MI355X): ", tcnn_last_error());
			nctx = c10::make_intrusive<NativeCtx>(c);
		}
		ctx->saved_data["module"] = module;
		ctx->saved_data["native"] = nctx;
		ctx->saved_data["loss_scale"] = loss_scale;
		ctx->save_for_backward({input, params, out});
		return out;
	}

	static torch::autograd::variable_list backward(torch::autograd::AutogradContext* ctx, torch::autograd::variable_list grads) {
		torch::Tensor doutput = grads[0];
		torch::autograd::variable_list none(4);
		if (!doutput.defined()) return none;
		TORCH_CHECK(doutput.is_cuda(), "tinycudann: doutput must be a GPU tensor");
		const auto saved = ctx->get_saved_variables();
		const torch::Tensor input = saved[0], params = saved[1], output = saved[2];
		tcnn_module* m = module_of(ctx);
		const double ls = ctx->saved_data.at("loss_scale").toDouble();
		if (!torch::GradMode::is_enabled()) {
			// first order (no create_graph): one engine call -- doutput * loss_scale, Module::backward and the
			// division by loss_scale in the torch roundings (tcnn_module_backward_scaled)
			if (doutput.scalar_type() != output.scalar_type()) doutput = doutput.to(output.scalar_type());
			if (!doutput.is_contiguous()) doutput = doutput.contiguous();
			const int64_t B = input.size(0);
			// needs_input_grad counts the tensor arguments only: 0 = input, 1 = params
			torch::Tensor gin = ctx->needs_input_grad(0) ? torch::empty_like(input) : torch::Tensor();
			torch::Tensor gpar = ctx->needs_input_grad(1) ? torch::empty({(int64_t)tcnn_module_n_params(m)}, params.options()) : torch::Tensor();
			check(tcnn_module_backward_scaled(m, stream_of(input), native(ctx), (uint32_t)B, (float*)ptr(gin), ptr(doutput), ptr(gpar),
			                                  (const float*)ptr(input), ptr(output), ptr(params), (float)ls, 0));
			return {torch::Tensor(), gin, gpar, torch::Tensor()};
		}
		auto g = ModuleBackward::apply((int64_t)m, ctx->saved_data.at("native"), ls, doutput, input, params, output);
		auto nn = [](const torch::Tensor& t) { return t.dim() == 0 ? torch::Tensor() : t; };  // null_tensor_to_none
		return {torch::Tensor(), nn(g[0]), nn(g[1]), torch::Tensor()};
	}
};

torch::Tensor module_apply(int64_t module, torch::Tensor input, torch::Tensor params, double loss_scale) {
	return ModuleFunction::apply(module, input, params, loss_scale);
}

}  // namespace

TORCH_LIBRARY(tcnn_mi355x, m) { m.class_<NativeCtx>("NativeCtx"); }

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
	m.doc() = "tinycudann (MI355X) torch autograd node in C++ over the engine's C-ABI";
	m.def("module_apply", &module_apply, "tinycudann.Module forward with its C++ autograd node (handle, input, params, loss_scale)");
}
