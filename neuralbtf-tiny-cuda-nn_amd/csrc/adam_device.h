// adam_device.h -- per-parameter Adam update (reference optimizers/adam.h:47-119), shared by the
// standalone optimizer kernel (kernels.hip) and the optimizer epilogues fused into the grid
// backward (grid.hip). The fp32 gradient sum is rounded to fp16 first because the reference's
// gradient buffer is __half (trainer.h:327); nvcc's contraction points are explicit FMAs.
#pragma once

#include "kernels.h"

namespace tcnn_amd {

__device__ __forceinline__ float adam_bias_factor(const AdamArgs& a, uint32_t st) {
	return sqrtf(1.0f - powf(a.beta2, (float)st)) / (1.0f - powf(a.beta1, (float)st));
}

// Adam on register values of parameter i (fp32 gradient sum gsum); returns false when the
// parameter is skipped (reference adam.h:75-82: frozen class, or a zero non-matrix gradient).
__device__ __forceinline__ bool adam_core(const AdamArgs& a, uint32_t i, float gsum, _Float16& g16, float& w, float& m1, float& m2,
                                          uint32_t& step) {
	g16 = (_Float16)(gsum * a.grad_scale);
	// x / 2^k is exact, so a power-of-two loss scale (128) becomes a multiply
	float gradient = a.inv_loss_scale != 0.0f ? (float)g16 * a.inv_loss_scale : (float)g16 / a.loss_scale;
	if (i >= a.n_matrix) {
		if (!a.opt_nonmatrix || gradient == 0.0f) return false;
	} else {
		if (!a.opt_matrix) return false;
	}
	const float wfp = w;
	if (i < a.n_matrix) gradient = __builtin_fmaf(a.l2_reg, wfp, gradient);
	const float gsq = gradient * gradient;
	m1 = __builtin_fmaf(a.beta1, m1, (1.0f - a.beta1) * gradient);
	m2 = __builtin_fmaf(a.beta2, m2, (1.0f - a.beta2) * gsq);
	float lr = a.lr;
	if (i >= a.n_matrix) lr *= a.nonmat_lr_factor;
	const uint32_t st = ++step;
	lr *= (a.cached_factor && st == a.cached_step) ? *a.cached_factor : adam_bias_factor(a, st);
	const float eff = fminf(fmaxf(lr / (sqrtf(m2) + a.eps), a.lower_lr_bound), a.upper_lr_bound);
	const float decayed = __builtin_fmaf(1.0f - a.rel_decay * lr, wfp, -copysignf(a.abs_decay * lr, wfp));
	float nw = __builtin_fmaf(-eff, m1, decayed);
	if (a.clip != 0.0f) nw = fminf(fmaxf(nw, -a.clip), a.clip);
	w = nw;
	return true;
}

// Updates parameter i in memory; returns the parameter's fp16 value afterwards.
__device__ __forceinline__ _Float16 adam_update(const AdamArgs& a, const AdamBuffers& s, uint32_t i, float gsum) {
	float w = s.w32[i], m1 = s.m1[i], m2 = s.m2[i];
	uint32_t step = s.steps[i];
	_Float16 g16;
	const bool upd = adam_core(a, i, gsum, g16, w, m1, m2, step);
	if (s.g16) s.g16[i] = g16;
	if (!upd) return s.w16[i];
	s.w32[i] = w;
	s.m1[i] = m1;
	s.m2[i] = m2;
	s.steps[i] = step;
	const _Float16 h = (_Float16)w;
	s.w16[i] = h;
	return h;
}

// Fixed-order sum of n slab values src[j * stride], j = 0 .. n-1, with the loads issued 8 at a time
// (independent, so a wave keeps 8 HBM round trips in flight instead of one); the additions stay
// in order j = 0, 1, ... (bit-identical to a plain loop). T = float or f4.
template <typename T>
__device__ __forceinline__ T slab_sum(const T* src, size_t stride, uint32_t n) {
	T s = T{};
	for (uint32_t j0 = 0; j0 < n; j0 += 8) {
		T v[8];
#pragma unroll
		for (uint32_t u = 0; u < 8; ++u)
			if (j0 + u < n) v[u] = src[(j0 + u) * stride];
#pragma unroll
		for (uint32_t u = 0; u < 8; ++u)
			if (j0 + u < n) s += v[u];
	}
	return s;
}

// In-launch hand-off between workgroups (MI355X_MICROARCH.md "inter-workgroup visibility";
// cdna_hip_programming.md §6 Guideline 16, counter form): every wave drains its stores, lane 0 of
// the workgroup releases at agent scope and draws a ticket; the workgroup that draws n - 1 is the
// reducer and acquires before reading the others' slabs. The reducer resets the counter (counters
// are zeroed once at allocation). `flag` is a word of the caller's existing LDS array.
__device__ __forceinline__ bool arrive_last(uint32_t* counter, uint32_t n, volatile uint32_t* flag) {
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	if (threadIdx.x == 0) {
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		const uint32_t prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		const bool last = prev == n - 1;
		if (last) {
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			__hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
		*flag = last ? 1u : 0u;
	}
	__syncthreads();
	return *flag != 0;
}

}  // namespace tcnn_amd
