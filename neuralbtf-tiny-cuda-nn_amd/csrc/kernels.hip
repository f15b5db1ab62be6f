// kernels.hip -- gfx950 kernels of the hot path + their launchers: reductions, optimizer, loss.
// (fused grid+MLP kernels: fused.hip / mlp_fused.h; grid kernels: grid.hip)
//
//   k_reduce_partials   sum of per-workgroup fp32 partial slabs
//   k_adam              Adam (reference optimizers/adam.h:47-119) reading fp32 gradient sums
//   k_relative_l2       standalone RelativeL2 (reference losses/relative_l2.h:40-76)
#include "kernels.h"

#include <cstdlib>

#include "adam_device.h"
#include "grid_device.h"
#include "mlp_fused.h"

namespace tcnn_amd {
// =============================================================================================
// reductions, Adam, casts, loss
// =============================================================================================

// Sum of fp32 partial slabs, at most two deterministic passes: (param block, part group) -> group
// sums, then groups -> out. Every thread issues 4-wide loads over one group of parts.
__global__ __launch_bounds__(256) void k_reduce_groups(const float* __restrict__ in, uint32_t n_parts, uint32_t group,
                                                        uint32_t stride, uint32_t n, float* __restrict__ out, uint32_t out_stride) {
	const uint32_t p4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
	if (p4 >= n) return;
	const uint32_t j0 = blockIdx.y * group;
	const uint32_t j1 = min(n_parts, j0 + group);
	float* dst = out + (size_t)blockIdx.y * out_stride;
	if (p4 + 4 <= n && (stride % 4) == 0 && (out_stride % 4) == 0) {
		f4 s = {0.0f, 0.0f, 0.0f, 0.0f};
		s = slab_sum((const f4*)(in + (size_t)j0 * stride + p4), stride / 4, j1 - j0);
		*(f4*)(dst + p4) = s;
	} else {
		for (uint32_t p = p4; p < n && p < p4 + 4; ++p) {
			float s = 0.0f;
			s = slab_sum(in + (size_t)j0 * stride + p, stride, j1 - j0);
			dst[p] = s;
		}
	}
}

// fin.out: the sum goes out finalised for the torch binding (grad_finalize_store) instead of as fp32
__global__ __launch_bounds__(256) void k_grid_slab_reduce(const float* __restrict__ in, uint32_t n_parts, uint32_t stride, uint32_t n,
                                                           float* __restrict__ out, const GridSlabMap* __restrict__ map, GradFinalize fin) {
	const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
	if (p >= n) return;
	const float s = slab_sum(in + (map ? grid_slab_index(map, p) : p), stride, n_parts);
	if (fin.out) grad_finalize_store(s, fin.s, fin.out, p, fin.out_f32);
	else out[p] = s;
}

void launch_grid_slab_reduce(hipStream_t st, const float* in, uint32_t n_parts, uint32_t stride, uint32_t n, float* out,
                             const GridSlabMap* map, GradFinalize fin) {
	if (!n) return;
	hipLaunchKernelGGL(k_grid_slab_reduce, dim3(div_round_up(n, 256)), dim3(256), 0, st, in, n_parts, stride, n, out, map, fin);
	TCNN_HIP_CHECK(hipGetLastError());
}

__global__ __launch_bounds__(1024) void k_column_sums(const float* __restrict__ in, uint32_t n_parts, uint32_t N, uint32_t G,
                                                      float* __restrict__ out) {
	extern __shared__ float lds_cs[];
	const uint32_t cb = column_block(N, G);
	const uint32_t c0 = blockIdx.x * cb;
	if (c0 >= N) return;
	const uint32_t ncol = min(cb, N - c0);
	block_column_sums(in, n_parts, N, c0, ncol, lds_cs + cb, lds_cs);
	for (uint32_t t = threadIdx.x; t < ncol; t += blockDim.x) out[c0 + t] = lds_cs[t];
}

uint32_t mlp_tail_groups() {
	static const uint32_t g = [] {
		const char* e = std::getenv("TCNN_MLP_TAIL_GROUPS");
		const int v = e ? std::atoi(e) : 0;
		return v > 0 && v <= 64 ? (uint32_t)v : 16u;
	}();
	return g;
}

void launch_column_sums(hipStream_t st, const float* in, uint32_t n_parts, uint32_t N, float* out) {
	TCNN_CHECK(N % 4 == 0, "column sums: N must be a multiple of 4");
	if (!N) return;
	const uint32_t G = mlp_tail_groups(), cb = column_block(N, G);
	const uint32_t S = std::max(1u, 1024u / (cb / 4));
	const size_t lds = (size_t)(cb + S * cb) * 4;
	TCNN_CHECK(lds <= 64 * 1024, "column sums: column block too large");
	hipLaunchKernelGGL(k_column_sums, dim3(G), dim3(1024), lds, st, in, n_parts, N, G, out);
	TCNN_HIP_CHECK(hipGetLastError());
}

size_t reduce_partials_tmp_floats(uint32_t n_parts, uint32_t n) {
	constexpr uint32_t MAXG = 16;
	if (n_parts <= MAXG) return 0;
	const uint32_t group = div_round_up(n_parts, MAXG);
	return (size_t)div_round_up(n_parts, group) * ((n + 3) / 4 * 4);
}

void launch_reduce_partials(hipStream_t st, const float* in, uint32_t n_parts, uint32_t stride, uint32_t n, float* out, float* tmp) {
	if (n == 0) return;
	constexpr uint32_t MAXG = 16;
	const uint32_t bx = div_round_up(div_round_up(n, 4), 256);
	if (n_parts <= MAXG) {
		hipLaunchKernelGGL(k_reduce_groups, dim3(bx, 1), dim3(256), 0, st, in, n_parts, n_parts, stride, n, out, 0u);
	} else {
		const uint32_t group = div_round_up(n_parts, MAXG);
		const uint32_t G = div_round_up(n_parts, group);
		const uint32_t ostride = (n + 3) / 4 * 4;
		TCNN_CHECK(tmp != nullptr, "reduce partials: scratch missing");
		hipLaunchKernelGGL(k_reduce_groups, dim3(bx, G), dim3(256), 0, st, in, n_parts, group, stride, n, tmp, ostride);
		TCNN_HIP_CHECK(hipGetLastError());
		hipLaunchKernelGGL(k_reduce_groups, dim3(bx, 1), dim3(256), 0, st, tmp, G, G, ostride, n, out, 0u);
	}
	TCNN_HIP_CHECK(hipGetLastError());
}

// pcg32 (dependencies/pcg32/pcg32.h:53-69, 139-158): jump `delta` steps ahead, then next_float
__device__ __forceinline__ void pcg32_advance(uint64_t& state, uint64_t inc, uint64_t delta) {
	constexpr uint64_t MULT = 0x5851f42d4c957f2dULL;
	uint64_t cur_mult = MULT, cur_plus = inc, acc_mult = 1u, acc_plus = 0u;
	for (; delta > 0; delta >>= 1) {
		if (delta & 1u) {
			acc_mult *= cur_mult;
			acc_plus = acc_plus * cur_mult + cur_plus;
		}
		cur_plus = (cur_mult + 1u) * cur_plus;
		cur_mult *= cur_mult;
	}
	state = acc_mult * state + acc_plus;
}

__device__ __forceinline__ float pcg32_next_float(uint64_t& state, uint64_t inc) {
	const uint64_t old = state;
	state = old * 0x5851f42d4c957f2dULL + inc;
	const uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
	const uint32_t rot = (uint32_t)(old >> 59u);
	const uint32_t u = ((xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31))) >> 9 | 0x3f800000u;
	return __builtin_bit_cast(float, u) - 1.0f;
}

// generate_random_kernel<float, pcg32, 4> (random.h:39-55): thread i jumps 4 i steps and writes
// out[i + n_threads j], j < 4; value = fma(u, upper - lower, lower) (the transform of random.h:69)
__global__ __launch_bounds__(128) void k_generate_uniform(uint64_t n, uint64_t state, uint64_t inc, float* __restrict__ out, float lo, float range) {
	const uint64_t i = threadIdx.x + (uint64_t)blockIdx.x * blockDim.x;
	const uint64_t n_threads = (uint64_t)blockDim.x * gridDim.x;
	pcg32_advance(state, inc, i * 4);
#pragma unroll
	for (uint32_t j = 0; j < 4; ++j) {
		const uint64_t idx = i + n_threads * j;
		if (idx >= n) return;
		out[idx] = __builtin_fmaf(pcg32_next_float(state, inc), range, lo);
	}
}

// random.h:77-80 generate_random_logistic: logit(u) * stddev * 0.551328895 + mean over the same
// strided uniform stream (common_device.h:46-48 logit, its clamp to [1e-9, 1 - 1e-9])
__global__ __launch_bounds__(128) void k_generate_logistic(uint64_t n, uint64_t state, uint64_t inc, float* __restrict__ out, float mean,
                                                           float stddev) {
	const uint64_t i = threadIdx.x + (uint64_t)blockIdx.x * blockDim.x;
	const uint64_t n_threads = (uint64_t)blockDim.x * gridDim.x;
	pcg32_advance(state, inc, i * 4);
#pragma unroll
	for (uint32_t j = 0; j < 4; ++j) {
		const uint64_t idx = i + n_threads * j;
		if (idx >= n) return;
		const float u = pcg32_next_float(state, inc);
		const float l = -logf(1.0f / fminf(fmaxf(u, 1e-9f), 1.0f - 1e-9f) - 1.0f);
		out[idx] = __builtin_fmaf(l * stddev, 0.551328895f, mean);
	}
}

void launch_generate_logistic(hipStream_t st, uint64_t n, uint64_t state, uint64_t inc, float* out, float mean, float stddev) {
	if (n == 0) return;
	const uint64_t n_thr = (n + 3) / 4;
	hipLaunchKernelGGL(k_generate_logistic, dim3((uint32_t)((n_thr + 127) / 128)), dim3(128), 0, st, n, state, inc, out, mean, stddev);
	TCNN_HIP_CHECK(hipGetLastError());
}

// trainer.h:114-121: the perturbed output the loss sees, add<<<>>> (common_device.h:963-968)
__global__ void k_add_perturbation(uint32_t n, const _Float16* __restrict__ out, const float* __restrict__ noise, _Float16* __restrict__ pert) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) pert[i] = (_Float16)((float)out[i] + noise[i]);
}
void launch_add_perturbation(hipStream_t st, uint32_t n, const void* out16, const float* noise, void* pert16) {
	if (!n) return;
	hipLaunchKernelGGL(k_add_perturbation, dim3(div_round_up(n, 256u)), dim3(256), 0, st, n, (const _Float16*)out16, noise, (_Float16*)pert16);
	TCNN_HIP_CHECK(hipGetLastError());
}

void launch_generate_uniform(hipStream_t st, uint64_t n, uint64_t state, uint64_t inc, float* out, float lo, float hi) {
	if (n == 0) return;
	const uint64_t n_thr = (n + 3) / 4;
	hipLaunchKernelGGL(k_generate_uniform, dim3((uint32_t)((n_thr + 127) / 128)), dim3(128), 0, st, n, state, inc, out, lo, hi - lo);
	TCNN_HIP_CHECK(hipGetLastError());
}


// reference optimizers/adam.h:47-119 (per-parameter update in adam_device.h)
__global__ __launch_bounds__(256) void k_adam(const AdamArgs a, float* __restrict__ w32, _Float16* __restrict__ w16,
                                               const float* __restrict__ grad32, _Float16* __restrict__ grad16,
                                               float* __restrict__ m1, float* __restrict__ m2, uint32_t* __restrict__ steps) {
	const uint32_t i = a.begin + blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= a.n) return;
	float gsum;
	if (a.part) {
		const uint32_t q = a.part_map ? grid_slab_index(a.part_map, i - a.begin) : i - a.begin;
		gsum = slab_sum(a.part + q, a.part_stride, a.n_parts);
		((float*)grad32)[i] = gsum;
	} else {
		gsum = grad32[i];
	}
	const AdamBuffers s{w32, w16, (float*)grad32, grad16, m1, m2, steps};
	adam_update(a, s, i, gsum);
}

void launch_adam(hipStream_t st, const AdamArgs& a, float* w32, void* w16, const float* grad32, void* grad16,
                 float* m1, float* m2, uint32_t* steps) {
	if (a.n <= a.begin) return;
	// one parameter per thread: measured faster than 4-wide vector access (16.7 vs 19.5 us for the
	// config_hash grid range with 8 slabs) -- 4x the waves in flight for the slab loads; r06 again with
	// the slabs in parameter order (16-byte slab and state loads): 9.3 vs 8.7 us at 2^15, 13.5 vs 13.0 at 2^18
	hipLaunchKernelGGL(k_adam, dim3(div_round_up(a.n - a.begin, 256)), dim3(256), 0, st, a, w32, (_Float16*)w16, grad32, (_Float16*)grad16, m1, m2, steps);
	TCNN_HIP_CHECK(hipGetLastError());
}

__global__ void k_cast_f32_f16(const float* __restrict__ in, _Float16* __restrict__ out, size_t n) {
	const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) out[i] = (_Float16)in[i];
}
__global__ void k_cast_f16_f32(const _Float16* __restrict__ in, float* __restrict__ out, size_t n) {
	const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) out[i] = (float)in[i];
}
// The torch binding's loss-scale arithmetic (reference bindings/torch/tinycudann/modules.py:128-137) done
// by the engine, in torch's rounding: fp16 x scalar and fp16 / scalar compute in fp32 and round once
// to fp16 (f16_rn: no fused mix rounding), fp32 / scalar in fp32.
__global__ void k_scale_f16(const _Float16* __restrict__ in, _Float16* __restrict__ out, float s, size_t n) {
	const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) out[i] = f16_rn((float)in[i] * s);
}
__global__ void k_div_f32(float* __restrict__ x, float s, size_t n) {
	const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) x[i] = x[i] / s;
}
__global__ void k_div_f16(const _Float16* __restrict__ in, void* __restrict__ out, float s, size_t n, int out_f32) {
	const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const _Float16 h = f16_rn((float)in[i] / s);
	if (out_f32) ((float*)out)[i] = (float)h;
	else ((_Float16*)out)[i] = h;
}
// fp32 gradient sum -> the binding's parameter gradient fp16(fp16(g) / s): the module's fp16 gradient
// buffer (cast) divided by the loss scale in torch (fp16 / scalar), in one pass
__global__ void k_grad_finalize(const float* __restrict__ g, void* __restrict__ out, float s, size_t n, int out_f32) {
	const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	grad_finalize_store(g[i], s, out, i, out_f32);
}
void launch_grad_finalize(hipStream_t st, const float* g, void* out, float s, size_t n, bool out_f32) {
	if (!n) return;
	hipLaunchKernelGGL(k_grad_finalize, dim3(div_round_up(n, 256)), dim3(256), 0, st, g, out, s, n, out_f32 ? 1 : 0);
	TCNN_HIP_CHECK(hipGetLastError());
}

void launch_scale_f16(hipStream_t st, const void* in, void* out, float s, size_t n) {
	if (!n) return;
	hipLaunchKernelGGL(k_scale_f16, dim3(div_round_up(n, 256)), dim3(256), 0, st, (const _Float16*)in, (_Float16*)out, s, n);
	TCNN_HIP_CHECK(hipGetLastError());
}
void launch_div_f32(hipStream_t st, float* x, float s, size_t n) {
	if (!n) return;
	hipLaunchKernelGGL(k_div_f32, dim3(div_round_up(n, 256)), dim3(256), 0, st, x, s, n);
	TCNN_HIP_CHECK(hipGetLastError());
}
void launch_div_f16(hipStream_t st, const void* in, void* out, float s, size_t n, bool out_f32) {
	if (!n) return;
	hipLaunchKernelGGL(k_div_f16, dim3(div_round_up(n, 256)), dim3(256), 0, st, (const _Float16*)in, out, s, n, out_f32 ? 1 : 0);
	TCNN_HIP_CHECK(hipGetLastError());
}

void launch_cast_f32_f16(hipStream_t st, const float* in, void* out, size_t n) {
	if (!n) return;
	hipLaunchKernelGGL(k_cast_f32_f16, dim3(div_round_up(n, 256)), dim3(256), 0, st, in, (_Float16*)out, n);
	TCNN_HIP_CHECK(hipGetLastError());
}
void launch_cast_f16_f32(hipStream_t st, const void* in, float* out, size_t n) {
	if (!n) return;
	hipLaunchKernelGGL(k_cast_f16_f32, dim3(div_round_up(n, 256)), dim3(256), 0, st, (const _Float16*)in, out, n);
	TCNN_HIP_CHECK(hipGetLastError());
}

__global__ __launch_bounds__(256) void k_relative_l2(uint32_t n_elements, uint32_t stride, uint32_t dims, float loss_scale,
                                                      const _Float16* __restrict__ pred, const float* __restrict__ target,
                                                      float* __restrict__ values, _Float16* __restrict__ grads) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n_elements) return;
	const uint32_t intra = i % stride, inter = i / stride;
	if (intra >= dims) {
		if (values) values[i] = 0.0f;
		grads[i] = (_Float16)0.0f;
		return;
	}
	const float n_total = (float)(n_elements / stride * dims);
	const float p = (float)pred[i];
	const float pse = __builtin_fmaf(p, p, 0.01f);
	const float d = p - target[inter * dims + intra];
	if (values) values[i] = d * d / pse / n_total;
	const float gr = 2.0f * d / pse;
	grads[i] = f16_rn(loss_scale * gr / n_total);
}

void launch_relative_l2(hipStream_t st, uint32_t B, uint32_t stride, uint32_t dims, float loss_scale,
                        const void* pred16, const float* target, float* values, void* grads16) {
	const uint32_t n = B * stride;
	if (!n) return;
	hipLaunchKernelGGL(k_relative_l2, dim3(div_round_up(n, 256)), dim3(256), 0, st, n, stride, dims, loss_scale,
	                   (const _Float16*)pred16, target, values, (_Float16*)grads16);
	TCNN_HIP_CHECK(hipGetLastError());
}

__global__ __launch_bounds__(256) void k_add_f32(const float* __restrict__ in, float* __restrict__ out, size_t n) {
	const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
	if (i < n) out[i] += in[i];
}

void launch_add_f32(hipStream_t st, const float* in, float* out, size_t n) {
	if (!n) return;
	hipLaunchKernelGGL(k_add_f32, dim3((uint32_t)div_round_up(n, 256)), dim3(256), 0, st, in, out, n);
	TCNN_HIP_CHECK(hipGetLastError());
}

__global__ __launch_bounds__(256) void k_sum(const float* __restrict__ in, uint32_t n, float* __restrict__ out) {
	__shared__ float part[4];
	float s = 0.0f;
	for (uint32_t i = threadIdx.x; i < n; i += 256) s += in[i];
#pragma unroll
	for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
	if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
	__syncthreads();
	if (threadIdx.x == 0) out[0] = part[0] + part[1] + part[2] + part[3];
}

void launch_sum(hipStream_t st, const float* in, uint32_t n, float* out) {
	hipLaunchKernelGGL(k_sum, dim3(1), dim3(256), 0, st, in, n, out);
	TCNN_HIP_CHECK(hipGetLastError());
}

// =============================================================================================
// layout probe (MFMA f16 operand maps + ds_read_b64_tr_b16), checked by tests/test_gpu_probe.py
// =============================================================================================
__global__ void k_probe(float* mfma_out, int16_t* tr_out) {
	extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
	uint16_t* S = (uint16_t*)smem;
	const int l = threadIdx.x, c = l & 15, q = l >> 4;
	for (int j = l; j < 32 * 24; j += 64) S[j] = (uint16_t)((j / 24) * 64 + (j % 24));
	__syncthreads();
	h8 av, bv;
	for (int e = 0; e < 8; ++e) {
		const int k = 8 * q + e;
		av[e] = (_Float16)(float)(((c * 3 + k * 5) % 11) - 5);  // A[i=c][k]
		bv[e] = (_Float16)(float)(((k * 7 + c * 2) % 13) - 6);  // B[k][j=c]
	}
	const f4 d = mfma16(av, bv, f4{0.0f, 0.0f, 0.0f, 0.0f});
	for (int r = 0; r < 4; ++r) mfma_out[l * 4 + r] = d[r];
	const h8 t = lds_trfrag(smem, 24, q, c, 0);
	*(uint4*)(tr_out + l * 8) = __builtin_bit_cast(uint4, t);
}

__global__ void k_probe_hfma(const h2* a, const h2* b, const h2* c, h2* out, uint32_t n) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) out[i] = pk_fma_f16(a[i], b[i], c[i]);
}

void launch_probe_hfma(hipStream_t st, const void* a, const void* b, const void* c, void* out, uint32_t n_pairs) {
	hipLaunchKernelGGL(k_probe_hfma, dim3(div_round_up(n_pairs, 256)), dim3(256), 0, st, (const h2*)a, (const h2*)b, (const h2*)c, (h2*)out, n_pairs);
	TCNN_HIP_CHECK(hipGetLastError());
}

void launch_probe(hipStream_t st, float* mfma_out, int16_t* tr_out) {
	hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 32 * 24 * 2, st, mfma_out, tr_out);
	TCNN_HIP_CHECK(hipGetLastError());
}

}  // namespace tcnn_amd
