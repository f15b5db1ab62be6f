// A caller written against the reference's tcnn::cpp API (cpp_api.h), built against this engine's
// include/tiny-cuda-nn/cpp_api.h + libtcnn_mi355x.so. Run on a GPU it trains nothing; it checks
// forward/backward/second-order calls through the Module interface and prints "cpp_api ok".
#include <tiny-cuda-nn/cpp_api.h>

#include <cmath>
#include <cstdio>
#include <vector>

int main() {
	using namespace tcnn::cpp;
	const json enc = {{"otype", "HashGrid"}, {"n_levels", 8}, {"n_features_per_level", 2}, {"log2_hashmap_size", 15},
	                  {"base_resolution", 16}, {"per_level_scale", 1.5}};
	const json net = {{"otype", "FullyFusedMLP"}, {"activation", "ReLU"}, {"output_activation", "None"},
	                  {"n_neurons", 64}, {"n_hidden_layers", 2}};
	std::unique_ptr<Module> model{create_network_with_input_encoding(2, 3, enc, net)};
	std::unique_ptr<Module> grid{create_encoding(2, enc, preferred_precision())};
	const uint32_t n = batch_size_granularity() * 4;
	if (model->n_output_dims() != 16 || model->param_precision() != Precision::Fp16 || default_loss_scale(Precision::Fp16) != 128.0f) {
		std::printf("unexpected module properties\n");
		return 1;
	}
	float *x, *p32, *dx, *ddx;
	void *p16, *out, *dy, *g16, *gp16, *gout, *ggrad;
	(void)hipMalloc(&x, n * 2 * 4);
	(void)hipMalloc(&dx, n * 2 * 4);
	(void)hipMalloc(&ddx, n * 2 * 4);
	(void)hipMalloc(&p32, model->n_params() * 4);
	(void)hipMalloc(&p16, model->n_params() * 2);
	(void)hipMalloc(&out, n * 16 * 2);
	(void)hipMalloc(&dy, n * 16 * 2);
	(void)hipMalloc(&g16, model->n_params() * 2);
	(void)hipMalloc(&gp16, grid->n_params() * 2);
	(void)hipMalloc(&gout, n * grid->n_output_dims() * 2);
	(void)hipMalloc(&ggrad, grid->n_params() * 2);
	std::vector<float> hx(n * 2);
	for (uint32_t i = 0; i < n * 2; ++i) hx[i] = std::fmod(0.618034f * (float)i, 1.0f);
	(void)hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
	(void)hipMemcpy(ddx, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
	(void)hipMemset(dy, 0, n * 16 * 2);
	(void)hipMemset(p16, 0, model->n_params() * 2);
	(void)hipMemset(gp16, 0, grid->n_params() * 2);
	model->initialize_params(1337, p32);
	hipStream_t st;
	(void)hipStreamCreate(&st);
	model->inference(st, n, x, out, p16);
	Context ctx = model->forward(st, n, x, out, p16, true);
	model->backward(st, ctx, n, dx, dy, g16, x, out, p16);
	Context gctx = grid->forward(st, n, x, gout, gp16, true);
	grid->backward_backward_input(st, gctx, n, ddx, x, gout, ggrad, nullptr, dx, gp16);
	bool threw = false;
	try {
		model->backward_backward_input(st, ctx, n, ddx, x, dy, g16, nullptr, dx, p16);
	} catch (const std::runtime_error&) {
		threw = true;  // networks have no second-order gradients (object.h:278-288)
	}
	if (hipStreamSynchronize(st) != hipSuccess || !threw) {
		std::printf("failed\n");
		return 1;
	}
	std::printf("cpp_api ok: %s / %s, %zu + %zu params, hyperparams otype %s\n", model->name().c_str(), grid->name().c_str(),
	            model->n_params(), grid->n_params(), model->hyperparams()["otype"].get<std::string>().c_str());
	return 0;
}
