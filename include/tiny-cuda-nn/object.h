// tiny-cuda-nn/object.h -- DifferentiableObject<T, PARAMS_T, COMPUTE_T> (reference
// include/tiny-cuda-nn/object.h:116-288) for the MI355X engine: the model interface the Trainer
// trains (trainer.h:50). Models here describe themselves to the engine -- the encoding and network
// configuration the engine builds (engine_encoding / engine_network) -- and run on the parameters of
// the Trainer that owns them (attach), like the reference's objects whose parameter pointers the
// Trainer sets (trainer.h:322-336). Implemented by NetworkWithInputEncoding<T>
// (network_with_input_encoding.h), Network<T, PARAMS_T> (network.h: the network alone, an Identity
// encoding in engine terms) and Encoding<T> (encoding.h).
#pragma once

#include <string>

#include "gpu_matrix.h"

namespace tcnn {

namespace detail {
// fp16 -> fp32 (the engine's inputs are fp32; a Network<__half> takes fp16 inputs, object.h:147)
template <typename T>
__global__ void widen_to_float(uint32_t n, const T* __restrict__ in, float* __restrict__ out) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) out[i] = (float)in[i];
}
template <typename T>
__global__ void narrow_from_float(uint32_t n, const float* __restrict__ in, T* __restrict__ out) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) out[i] = (T)in[i];
}
// the engine's fp32 view of an input matrix: the matrix itself, or a widened copy in `scratch`
template <typename T>
inline const float* engine_input(hipStream_t stream, const GPUMatrixDynamic<T>& input, GPUMemory<float>& scratch) {
	if constexpr (std::is_same<T, float>::value) {
		(void)stream;
		(void)scratch;
		return input.data();
	} else {
		const uint32_t n = (uint32_t)input.n_elements();
		scratch.enlarge(n);
		if (n) hipLaunchKernelGGL(widen_to_float<T>, dim3((n + 255) / 256), dim3(256), 0, stream, n, input.data(), scratch.data());
		return scratch.data();
	}
}
}  // namespace detail

template <typename T, typename PARAMS_T, typename COMPUTE_T = T>
class DifferentiableObject {
public:
	virtual ~DifferentiableObject() = default;

	virtual uint32_t input_width() const = 0;
	virtual uint32_t output_width() const = 0;
	virtual uint32_t padded_output_width() const = 0;
	virtual size_t n_params() const = 0;
	virtual json hyperparams() const = 0;
	virtual std::string name() const = 0;

	// what the engine builds for this model: the encoding and network configuration ({"otype":
	// "Identity"} for a network alone; a null network for an encoding alone)
	virtual json engine_encoding() const = 0;
	virtual json engine_network() const = 0;

	// set by the Trainer that owns this object's parameters
	void attach(tcnn_trainer* t) { m_trainer = t; }
	tcnn_trainer* trainer_handle() const { return m_trainer; }

	// object.h:147-179: output fp32 [output_width() x n] from input [input_width() x n], n a multiple
	// of 256, on the owning trainer's parameters
	void inference(hipStream_t stream, const GPUMatrixDynamic<T>& input, GPUMatrixDynamic<float>& output, bool use_inference_params = true) {
		(void)use_inference_params;  // one parameter set: the trainer's fp16 parameters
		CHECK_THROW(input.m() == input_width());
		CHECK_THROW(output.m() == output_width());
		CHECK_THROW(input.n() % BATCH_SIZE_GRANULARITY == 0);
		CHECK_THROW(input.n() == output.n());
		CHECK_THROW(input.layout() == CM && input.is_contiguous() && output.layout() == CM && output.is_contiguous());
		if (!m_trainer) {
			if (inference_standalone(stream, input, output)) return;
			throw std::runtime_error{name() + "::inference: no parameters (the object is not owned by a Trainer)"};
		}
		const float* in = detail::engine_input(stream, input, m_input_scratch);
		detail::check_rc(tcnn_trainer_inference(m_trainer, stream, input.n(), in, output.data()));
	}
	void inference(const GPUMatrixDynamic<T>& input, GPUMatrixDynamic<float>& output, bool use_inference_params = true) {
		inference(nullptr, input, output, use_inference_params);
	}

protected:
	// an object that holds its own parameters (Encoding) runs inference without a Trainer
	virtual bool inference_standalone(hipStream_t, const GPUMatrixDynamic<T>&, GPUMatrixDynamic<float>&) { return false; }
	tcnn_trainer* m_trainer = nullptr;
	GPUMemory<float> m_input_scratch;
};

}  // namespace tcnn
