// A caller of the reference's C++ template API (reference include/tiny-cuda-nn/config.h:46-63,
// trainer.h:163-211, object.h:147-179, gpu_matrix.h, gpu_memory.h, random.h, common_device.h:331),
// built against include/tiny-cuda-nn/*.h + libtcnn_mi355x.so and run by
// tests/test_gpu_template_api.py. Every check prints "FAIL ..." and exits nonzero on mismatch.
#include <tiny-cuda-nn/common_device.h>

#include <tiny-cuda-nn/config.h>
#include <tiny-cuda-nn/multi_stream.h>

#include <cmath>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <vector>

using namespace tcnn;

static int g_fail = 0;
#define EXPECT(c)                                                           \
	do {                                                                    \
		if (!(c)) {                                                         \
			std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);        \
			++g_fail;                                                       \
		}                                                                   \
	} while (0)

__global__ void field(uint32_t n, const float* __restrict__ xy, float* __restrict__ rgb) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const float x = xy[2 * i], y = xy[2 * i + 1];
	rgb[3 * i + 0] = 0.5f + 0.5f * sinf(9.0f * x) * cosf(7.0f * y);
	rgb[3 * i + 1] = 0.5f + 0.4f * sinf(23.0f * x * y + 1.0f);
	rgb[3 * i + 2] = 0.5f + 0.3f * cosf(31.0f * x) * sinf(17.0f * y);
}

__global__ void field16(uint32_t n, const __half* __restrict__ x, float* __restrict__ y) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	for (int k = 0; k < 3; ++k) y[3 * i + k] = 0.5f + 0.4f * sinf(3.0f * (float)x[16 * i + k] + 2.0f * (float)x[16 * i + k + 3]);
}

int main(int argc, char** argv) {
	if (argc < 2) {
		std::printf("usage: %s <config_hash.json>\n", argv[0]);
		return 2;
	}
	try {
		std::ifstream f{argv[1]};
		const json config = json::parse(std::string{std::istreambuf_iterator<char>{f}, std::istreambuf_iterator<char>{}});

		// default_rng_t == pcg32: known answers of the reference's own pcg32.h compiled in the build
		// container (tests/golden/ref_known_answers.json: pcg32_1337_next_uint / _next_float,
		// pcg32_1337_advance_1000003_next_uint)
		{
			default_rng_t r{1337};
			EXPECT(r.next_uint() == 634364130u);
			EXPECT(r.next_float() == 0.471029401f);
			default_rng_t a{1337};
			a.advance(1000003);
			EXPECT(a.next_uint() == 2652094483u);
		}
		// generate_random_uniform: device batch == host evaluation of the strided order, rng advanced by n
		{
			const uint32_t n = 1000;
			default_rng_t rng{1337};
			GPUMemory<float> buf(n);
			generate_random_uniform<float>(nullptr, rng, n, buf.data(), -2.0f, 3.0f);
			std::vector<float> got(n);
			buf.copy_to_host(got);
			const uint32_t n_thr = (n + 3) / 4, n_threads = (n_thr + 127) / 128 * 128;
			default_rng_t base{1337};
			int bad = 0;
			for (uint32_t i = 0; i < n_threads; ++i) {  // every launched thread writes (random.h:41-54)
				default_rng_t r = base;
				r.advance(4 * i);
				for (uint32_t j = 0; j < 4; ++j) {
					const uint32_t idx = i + n_threads * j;
					if (idx >= n) break;
					if (got[idx] != std::fma(r.next_float(), 5.0f, -2.0f)) ++bad;
				}
			}
			EXPECT(bad == 0);
			default_rng_t adv{1337};
			adv.advance(n);
			EXPECT(rng == adv);
		}
		// GPUMatrix conventions (gpu_matrix.h): m = features, n = batch, CM default
		{
			GPUMatrix<float> a(3, 512);
			EXPECT(a.m() == 3 && a.n() == 512 && a.layout() == CM && a.stride() == 3 && a.n_elements() == 1536);
			GPUMatrix<float> v(a.data(), 3, 512);
			EXPECT(v.data() == a.data());
			auto t = a.transposed();
			EXPECT(t.m() == 512 && t.n() == 3 && t.layout() == RM);
		}
		// workspace arena (gpu_memory.h:426-754): addresses survive growth, contents too; aligned
		// distribution; intervals are reused after free; SyncedMultiStream fork / join (multi_stream.h)
		{
			hipStream_t s;
			HIP_CHECK_THROW(hipStreamCreate(&s));
			uint64_t mapped0 = 0;
			int vmm = 0;
			{
				auto a = allocate_workspace(s, 1000);
				EXPECT(a.data() != nullptr && ((uintptr_t)a.data() % 128) == 0);
				HIP_CHECK_THROW(hipMemsetAsync(a.data(), 0x5a, 1000, s));
				tcnn_workspace_arena_info(s, &mapped0, &vmm);
				uint8_t* p0 = a.data();
				auto big = allocate_workspace(s, (size_t)3 << 30);  // grows the arena by 3 GiB
				uint64_t mapped1 = 0;
				tcnn_workspace_arena_info(s, &mapped1, &vmm);
				EXPECT(mapped1 >= ((uint64_t)3 << 30) && big.data() != nullptr);
				EXPECT(a.data() == p0);  // the first allocation did not move
				std::vector<uint8_t> h(1000);
				HIP_CHECK_THROW(hipMemcpyAsync(h.data(), a.data(), 1000, hipMemcpyDeviceToHost, s));
				HIP_CHECK_THROW(hipStreamSynchronize(s));
				bool kept = true;
				for (uint8_t v : h) kept = kept && v == 0x5a;
				EXPECT(kept);
				GPUMemoryArena::Allocation d;
				float* f;
				uint16_t* u;
				double* x;
				std::tie(f, u, x) = allocate_workspace_and_distribute<float, uint16_t, double>(s, &d, 3, 5, 7);
				EXPECT(((uintptr_t)f % 128) == 0 && ((uintptr_t)u % 128) == 0 && ((uintptr_t)x % 128) == 0);
				EXPECT((uint8_t*)u - (uint8_t*)f == 128 && (uint8_t*)x - (uint8_t*)u == 128);
			}
			{
				auto r = allocate_workspace(s, 1000);  // everything was freed: the first interval again
				EXPECT(r.data() != nullptr);
			}
			free_gpu_memory_arena(s);
			std::printf("arena vmm=%d\n", vmm);
			// growth while the stream is being captured (the reference defers its synchronisation to the
			// capture, gpu_memory.h:596-601; the VMM arena needs none): the graph writes the new memory
			if (vmm) {
				hipGraph_t g;
				hipGraphExec_t ge;
				HIP_CHECK_THROW(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
				auto grown = allocate_workspace(s, (size_t)1 << 30);
				HIP_CHECK_THROW(hipMemsetAsync(grown.data(), 0x7b, 4096, s));
				HIP_CHECK_THROW(hipStreamEndCapture(s, &g));
				HIP_CHECK_THROW(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
				HIP_CHECK_THROW(hipGraphLaunch(ge, s));
				std::vector<uint8_t> h(4096);
				HIP_CHECK_THROW(hipMemcpyAsync(h.data(), grown.data(), 4096, hipMemcpyDeviceToHost, s));
				HIP_CHECK_THROW(hipStreamSynchronize(s));
				bool ok = true;
				for (uint8_t v : h) ok = ok && v == 0x7b;
				EXPECT(ok);
				HIP_CHECK_THROW(hipGraphExecDestroy(ge));
				HIP_CHECK_THROW(hipGraphDestroy(g));
			}
			// detaching an arena that still has a live allocation (free_gpu_memory_arena of the reference
			// drops its shared_ptr; the allocation keeps the arena alive and frees into it later)
			{
				auto live = allocate_workspace(s, 1 << 20);
				free_gpu_memory_arena(s);
				HIP_CHECK_THROW(hipMemsetAsync(live.data(), 0, 1 << 20, s));
				HIP_CHECK_THROW(hipStreamSynchronize(s));
				auto fresh = allocate_workspace(s, 1 << 20);  // a new arena for the same stream
				EXPECT(fresh.data() != nullptr && fresh.data() != live.data());
			}
			free_all_gpu_memory_arenas();
			// fork / join: four streams each fill a quarter, the parent reads the whole after the join
			GPUMemory<float> buf(4096);
			{
				SyncedMultiStream ms{s, 4};
				for (size_t k = 0; k < 4; ++k) HIP_CHECK_THROW(hipMemsetD32Async((hipDeviceptr_t)(buf.data() + 1024 * k), 0x3f800000u * (k % 2) + 0x40000000u * (1 - k % 2), 1024, ms.get(k)));
			}
			std::vector<float> hb(4096);
			HIP_CHECK_THROW(hipMemcpyAsync(hb.data(), buf.data(), 4096 * 4, hipMemcpyDeviceToHost, s));
			HIP_CHECK_THROW(hipStreamSynchronize(s));
			bool ok = true;
			for (size_t i = 0; i < 4096; ++i) ok = ok && hb[i] == ((i / 1024) % 2 ? 1.0f : 2.0f);
			EXPECT(ok);
			free_multi_streams(s);
			HIP_CHECK_THROW(hipStreamDestroy(s));
		}
		// create_from_config -> training_step / loss / inference (config.h:53-63)
		const uint32_t B = 1 << 16;
		TrainableModel model = create_from_config(2, 3, config);
		EXPECT(model.trainer->n_params() == 715536);
		EXPECT(model.network->padded_output_width() == 16 && model.network->input_width() == 2 && model.network->output_width() == 3);
		EXPECT(model.trainer->engine() == "fused");

		hipStream_t stream;
		HIP_CHECK_THROW(hipStreamCreate(&stream));
		default_rng_t rng{1337};
		GPUMatrix<float> batch(2, B), target(3, B);
		GPUMatrix<float> probe(2, 4096), probe_out(3, 4096);
		generate_random_uniform<float>(stream, rng, probe.n_elements(), probe.data());
		float first = 0.0f, last = 0.0f;
		for (int i = 0; i < 200; ++i) {
			generate_random_uniform<float>(stream, rng, batch.n_elements(), batch.data());
			linear_kernel(field, 0, stream, B, batch.data(), target.data());
			auto ctx = model.trainer->training_step(stream, batch, target);
			if (i == 0) first = model.trainer->loss(stream, *ctx);
			if (i == 199) last = model.trainer->loss(stream, *ctx);
			if (i == 198) {
				// the loss of any live context, not only the most recent step's (trainer.h:205-211)
				auto old = std::move(ctx);
				const float l198 = model.trainer->loss(stream, *old);
				auto ctx2 = model.trainer->training_step(stream, batch, target);
				EXPECT(model.trainer->loss(stream, *old) == l198);
				++i;
				last = model.trainer->loss(stream, *ctx2);
				EXPECT(last != l198);
			}
		}
		std::printf("loss first=%g last=%g\n", first, last);
		EXPECT(std::isfinite(first) && last < 0.5f * first);
		EXPECT(model.optimizer->step() == 200u);

		// Trainer::forward / backward halves (trainer.h:97-153): Accumulate doubles the gradient, an
		// external dL/dy equal to the loss's own gives the same gradient, dL/dinput is written
		{
			const size_t n = model.trainer->n_params();
			auto fwd = model.trainer->forward(stream, 128.0f, batch, target);
			model.trainer->backward(stream, *fwd, batch);
			std::vector<float> g1(n), g2(n), g3(n);
			HIP_CHECK_THROW(hipStreamSynchronize(stream));
			HIP_CHECK_THROW(hipMemcpy(g1.data(), tcnn_trainer_gradients_fp32(model.trainer->handle()), n * 4, hipMemcpyDeviceToHost));
			model.trainer->backward(stream, *fwd, batch, nullptr, false, GradientMode::Accumulate);
			HIP_CHECK_THROW(hipStreamSynchronize(stream));
			HIP_CHECK_THROW(hipMemcpy(g2.data(), tcnn_trainer_gradients_fp32(model.trainer->handle()), n * 4, hipMemcpyDeviceToHost));
			auto ext = model.trainer->forward(stream, 128.0f, batch, target, nullptr, false, false, &fwd->dL_doutput);
			model.trainer->backward(stream, *ext, batch);
			HIP_CHECK_THROW(hipStreamSynchronize(stream));
			HIP_CHECK_THROW(hipMemcpy(g3.data(), tcnn_trainer_gradients_fp32(model.trainer->handle()), n * 4, hipMemcpyDeviceToHost));
			GPUMatrix<float> dx(2, B);
			auto fwd_dx = model.trainer->forward(stream, 128.0f, batch, target, nullptr, false, true);
			model.trainer->backward(stream, *fwd_dx, batch, &dx);
			bool dbl = true, same = true;
			for (size_t k = 0; k < n; ++k) {
				dbl = dbl && g2[k] == 2.0f * g1[k];
				same = same && g3[k] == g1[k];
			}
			EXPECT(dbl && same);
			EXPECT(std::isfinite(model.trainer->loss(stream, *fwd)) && model.trainer->loss(stream, *ext) == 0.0f);
			const std::vector<float> dxh = dx.to_cpu_vector();
			float mx = 0.0f;
			for (float v : dxh) mx = std::fmax(mx, std::fabs(v));
			EXPECT(mx > 0.0f && std::isfinite(mx));
			// GradientMode::Ignore: dL/dinput again, the parameter gradients stay those of the last backward
			std::vector<float> g4(n), g5(n);
			HIP_CHECK_THROW(hipStreamSynchronize(stream));
			HIP_CHECK_THROW(hipMemcpy(g4.data(), tcnn_trainer_gradients_fp32(model.trainer->handle()), n * 4, hipMemcpyDeviceToHost));
			GPUMatrix<float> dx2(2, B);
			model.trainer->backward(stream, *fwd_dx, batch, &dx2, false, GradientMode::Ignore);
			HIP_CHECK_THROW(hipStreamSynchronize(stream));
			HIP_CHECK_THROW(hipMemcpy(g5.data(), tcnn_trainer_gradients_fp32(model.trainer->handle()), n * 4, hipMemcpyDeviceToHost));
			EXPECT(g4 == g5 && dx2.to_cpu_vector() == dxh);
		}

		model.network->inference(stream, probe, probe_out);
		HIP_CHECK_THROW(hipStreamSynchronize(stream));
		const std::vector<float> out = probe_out.to_cpu_vector();
		bool finite = true;
		for (float v : out) finite = finite && std::isfinite(v);
		EXPECT(finite);

		// hyper-parameters reach the engine (adam.h:200-210)
		model.optimizer->set_learning_rate(1e-3f);
		EXPECT(std::fabs(model.optimizer->learning_rate() - 1e-3f) < 1e-9f);
		model.trainer->update_hyperparams({{"optimizer", {{"learning_rate", 2e-3f}}}});
		EXPECT(std::fabs(model.trainer->hyperparams()["optimizer"]["learning_rate"].get<float>() - 2e-3f) < 1e-9f);
		// the loss type is fixed at construction: a change is refused, not silently ignored
		model.trainer->update_hyperparams({{"loss", {{"otype", "RelativeL2"}}}});
		bool refused = false;
		try {
			model.trainer->update_hyperparams({{"loss", {{"otype", "L2"}}}});
		} catch (const std::runtime_error&) {
			refused = true;
		}
		EXPECT(refused);

		// parameters: set_params_full_precision round trip, snapshot round trip
		std::vector<float> p(model.trainer->n_params());
		HIP_CHECK_THROW(hipMemcpy(p.data(), model.trainer->params_full_precision(), p.size() * 4, hipMemcpyDeviceToHost));
		auto snap = model.trainer->serialize_msgpack(true);
		// json serialize / deserialize with the reference's signatures (trainer.h:275-315)
		const json jsnap = model.trainer->serialize(true);
		EXPECT(jsnap["n_params"].get<uint64_t>() == model.trainer->n_params() && jsnap["params_type"] == "__half");
		EXPECT(jsnap["params_binary"]["bytes"].size() == model.trainer->n_params() * 2);
		EXPECT(jsnap["optimizer"]["first_moments_binary"]["bytes"].size() == model.trainer->n_params() * 4);
		TrainableModel other = create_from_config(2, 3, config);
		other.trainer->set_params_full_precision(p.data(), p.size());
		std::vector<float> q(p.size());
		HIP_CHECK_THROW(hipMemcpy(q.data(), other.trainer->params_full_precision(), q.size() * 4, hipMemcpyDeviceToHost));
		EXPECT(p == q);
		TrainableModel third = create_from_config(2, 3, config);
		third.trainer->deserialize_msgpack(snap);
		GPUMatrix<float> out3(3, 4096);
		third.network->inference(stream, probe, out3);
		HIP_CHECK_THROW(hipStreamSynchronize(stream));
		EXPECT(out3.to_cpu_vector() == out);
		{
			TrainableModel fourth = create_from_config(2, 3, config);
			fourth.trainer->deserialize(jsnap);
			GPUMatrix<float> out4(3, 4096);
			fourth.network->inference(stream, probe, out4);
			HIP_CHECK_THROW(hipStreamSynchronize(stream));
			EXPECT(out4.to_cpu_vector() == out);
			EXPECT(fourth.trainer->serialize_msgpack(true) == snap);  // the optimizer state came back too
		}

		// the reference's error behaviour: CHECK_THROW on a batch that is not a multiple of 256
		{
			GPUMatrix<float> bad_in(2, 300), bad_t(3, 300);
			bool threw = false;
			try {
				model.trainer->training_step(stream, bad_in, bad_t);
			} catch (const std::runtime_error&) {
				threw = true;
			}
			EXPECT(threw);
			threw = false;
			try {
				create_loss<network_precision_t>({{"otype", "Huber"}});
			} catch (const std::runtime_error&) {
				threw = true;
			}
			EXPECT(threw);
		}
		// a network that no Trainer owns has no parameters
		{
			NetworkWithInputEncoding<network_precision_t> lone(2, 3, config["encoding"], config["network"]);
			bool threw = false;
			try {
				lone.inference(stream, probe, probe_out);
			} catch (const std::runtime_error&) {
				threw = true;
			}
			EXPECT(threw);
		}
		// output perturbation (trainer.h:50-57, 114-123): logistic noise of scale sigma on the output the
		// loss sees; the generator is random.h:77-80 over the uniform stream
		{
			const uint32_t n = 1 << 12;
			GPUMemory<float> noise(n);
			default_rng_t r{7};
			generate_random_logistic<float>(stream, r, n, noise.data(), 0.0f, 1.0f);
			std::vector<float> hn(n);
			noise.copy_to_host(hn);
			default_rng_t adv{7};
			adv.advance(n);
			EXPECT(r == adv);
			const uint32_t n_thr = (n + 3) / 4, n_threads = (n_thr + 127) / 128 * 128;
			default_rng_t base{7};
			int bad = 0;
			for (uint32_t i = 0; i < n_threads; ++i) {
				default_rng_t q = base;
				q.advance(4 * i);
				for (uint32_t j = 0; j < 4; ++j) {
					const uint32_t idx = i + n_threads * j;
					if (idx >= n) break;
					const float u = q.next_float();
					const float l = -std::log(1.0f / std::fmin(std::fmax(u, 1e-9f), 1.0f - 1e-9f) - 1.0f);
					if (std::fabs(hn[idx] - l * 0.551328895f) > 1e-5f * (1.0f + std::fabs(l))) ++bad;
				}
			}
			EXPECT(bad == 0);

			std::shared_ptr<NetworkWithInputEncoding<network_precision_t>> pnet{
			    new NetworkWithInputEncoding<network_precision_t>(2, 3, config["encoding"], config["network"])};
			std::shared_ptr<Loss<network_precision_t>> pl{create_loss<network_precision_t>(config["loss"])};
			std::shared_ptr<Optimizer<network_precision_t>> po{create_optimizer<network_precision_t>(config["optimizer"])};
			Trainer<float, network_precision_t, network_precision_t> pt(pnet, po, pl, 1337, 0.05f);
			EXPECT(pt.perturbation_sigma() == 0.05f);
			float p0 = 0, p1 = 0;
			for (int i = 0; i < 100; ++i) {
				auto ctx = pt.training_step(stream, batch, target);
				if (i == 0) p0 = pt.loss(stream, *ctx);
				if (i == 99) p1 = pt.loss(stream, *ctx);
			}
			std::printf("perturbed training (sigma 0.05): loss %g -> %g\n", p0, p1);
			EXPECT(std::isfinite(p1) && p1 < 0.7f * p0);
			// the context keeps the unperturbed output: it equals inference on the same parameters
			auto fc = pt.forward(stream, 128.0f, probe, probe_out);
			GPUMatrix<float> inf(3, 4096);
			pnet->inference(stream, probe, inf);
			HIP_CHECK_THROW(hipStreamSynchronize(stream));
			std::vector<__half> o16(16 * 4096);
			HIP_CHECK_THROW(hipMemcpy(o16.data(), fc->output.data(), o16.size() * 2, hipMemcpyDeviceToHost));
			const std::vector<float> hi = inf.to_cpu_vector();
			int diff = 0;
			for (uint32_t i = 0; i < 4096; ++i)
				for (uint32_t k = 0; k < 3; ++k) diff += (float)o16[(size_t)i * 16 + k] != hi[(size_t)i * 3 + k];
			EXPECT(diff == 0);

			// initialize_params re-initialises from the trainer's live generator (trainer.h:67-85: m_rng
			// keeps advancing), so a second initialisation draws new values -- the first n_params draws
			// after the construction-time ones: the network's first weight equals the Xavier transform of
			// the generator advanced by n_params
			std::shared_ptr<NetworkWithInputEncoding<network_precision_t>> rnet{
			    new NetworkWithInputEncoding<network_precision_t>(2, 3, config["encoding"], config["network"])};
			Trainer<float, network_precision_t, network_precision_t> rt(rnet, po, pl, 1337);
			const uint64_t np = tcnn_trainer_n_params(rt.handle());
			std::vector<float> w0(np), w1(np);
			HIP_CHECK_THROW(hipMemcpy(w0.data(), tcnn_trainer_params_fp32(rt.handle()), np * 4, hipMemcpyDeviceToHost));
			rt.initialize_params();
			HIP_CHECK_THROW(hipMemcpy(w1.data(), tcnn_trainer_params_fp32(rt.handle()), np * 4, hipMemcpyDeviceToHost));
			std::seed_seq seq{1337u};
			std::vector<uint32_t> sd(2);
			seq.generate(sd.begin(), sd.end());
			default_rng_t g{sd.front()};
			g.advance((int64_t)np);
			const float scale = std::sqrt(6.0f / (float)(64 + 32));  // W0 of config_hash: 64 x 32
			volatile float t0 = g.next_float() * 2.0f;  // the engine's xavier: t = u * 2; t = t * scale; t - scale
			volatile float t1 = t0 * scale;
			const float x0 = t1 - scale;
			EXPECT(w1[0] == x0);
			EXPECT(w0[0] != w1[0]);
		}

		// Trainer over any DifferentiableObject (trainer.h:50): a Network alone from create_network
		// (network.h:141-158), fp16 inputs (Trainer<__half, __half, __half>), and an Encoding alone refused
		{
			const uint32_t n = 1 << 14;
			std::shared_ptr<Network<network_precision_t>> net{create_network<network_precision_t>(
			    {{"otype", "FullyFusedMLP"}, {"activation", "ReLU"}, {"output_activation", "None"}, {"n_neurons", 64},
			     {"n_hidden_layers", 2}, {"n_input_dims", 16}, {"n_output_dims", 3}})};
			EXPECT(net->input_width() == 16 && net->output_width() == 3 && net->width(1) == 64 && net->num_forward_activations() == 2);
			std::shared_ptr<Loss<network_precision_t>> l{create_loss<network_precision_t>({{"otype", "L2"}})};
			std::shared_ptr<Optimizer<network_precision_t>> o{
			    create_optimizer<network_precision_t>({{"otype", "Adam"}, {"learning_rate", 1e-2f}})};
			auto tr = std::make_shared<Trainer<network_precision_t, network_precision_t, network_precision_t>>(net, o, l);
			EXPECT(tr->n_params() == net->n_params() && net->n_params() == 64 * 16 + 64 * 64 + 16 * 64);
			GPUMemory<float> x32(16 * n);
			default_rng_t r{42};
			generate_random_uniform<float>(stream, r, 16 * n, x32.data(), -1.0f, 1.0f);
			GPUMatrix<network_precision_t> x(16, n);
			hipLaunchKernelGGL(detail::narrow_from_float<network_precision_t>, dim3(16 * n / 256), dim3(256), 0, stream, 16 * n,
			                   x32.data(), x.data());
			GPUMatrix<float> y(3, n);
			hipLaunchKernelGGL(field16, dim3(n / 256), dim3(256), 0, stream, n, x.data(), y.data());
			float l0 = 0, l1 = 0;
			for (int i = 0; i < 300; ++i) {
				auto ctx = tr->training_step(stream, x, y);
				if (i == 0) l0 = tr->loss(stream, *ctx);
				if (i == 299) l1 = tr->loss(stream, *ctx);
			}
			std::printf("create_network fp16 inputs: L2 %.5f -> %.5f\n", l0, l1);
			EXPECT(std::isfinite(l1) && l1 < 0.25f * l0);
			// inference on the trainer's parameters equals forward's output
			GPUMatrix<float> yi(3, n);
			net->inference(stream, x, yi);
			auto ctx = tr->forward(stream, 1.0f, x, y, nullptr, false, true);
			HIP_CHECK_THROW(hipStreamSynchronize(stream));
			EXPECT(std::isfinite(yi.to_cpu_vector()[0]));
			// dL/dinput narrowed to fp16 for a fp16-input trainer
			GPUMatrix<network_precision_t> dx(16, n);
			tr->backward(stream, *ctx, x, &dx, false, GradientMode::Ignore);
			HIP_CHECK_THROW(hipStreamSynchronize(stream));
			std::vector<network_precision_t> hdx(16 * n);
			HIP_CHECK_THROW(hipMemcpy(hdx.data(), dx.data(), hdx.size() * 2, hipMemcpyDeviceToHost));
			bool nonzero = false;
			for (auto v : hdx) nonzero = nonzero || (float)v != 0.0f;
			EXPECT(nonzero);

			std::shared_ptr<Encoding<network_precision_t>> enc{create_encoding<network_precision_t>(2, config["encoding"])};
			EXPECT(enc->input_width() == 2 && enc->output_width() == 32);
			// an Encoding holds its own (initialised) parameters: inference runs without a Trainer
			{
				GPUMatrix<float> eo(32, 4096);
				enc->inference(stream, probe, eo);
				HIP_CHECK_THROW(hipStreamSynchronize(stream));
				const std::vector<float> ev = eo.to_cpu_vector();
				float emax = 0.0f;
				bool efin = true;
				for (float v : ev) {
					efin = efin && std::isfinite(v);
					emax = std::fmax(emax, std::fabs(v));
				}
				EXPECT(efin && emax > 0.0f && emax <= 2e-4f);  // grid init: uniform in +-1e-4, weights sum to 1
			}
			bool refused = false;
			try {
				Trainer<float, network_precision_t, network_precision_t> bad(enc, o, l);
			} catch (const std::runtime_error&) {
				refused = true;
			}
			EXPECT(refused);
		}
		free_all_gpu_memory_arenas();
		HIP_CHECK_THROW(hipStreamDestroy(stream));
	} catch (const std::exception& e) {
		std::printf("FAIL exception: %s\n", e.what());
		return 1;
	}
	if (g_fail) return 1;
	std::printf("template api ok\n");
	return 0;
}
