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
	g16 = f16_rn(gsum * a.grad_scale);
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
	lr *= (st - 1u < a.factor_n) ? a.factor_table[st - 1u] : adam_bias_factor(a, st);
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
	const _Float16 h = f16_rn(w);
	s.w16[i] = h;
	return h;
}

// Adam state of 4 consecutive parameters (i % 4 == 0): one 16-byte load per state array, so a
// thread keeps 5 independent HBM round trips in flight instead of a chain of scalar ones.
struct AdamState4 {
	f4 w, m1, m2;
	uint4 st;
	h4 w16;
};

__device__ __forceinline__ AdamState4 adam_load4(const AdamBuffers& s, uint32_t i) {
	AdamState4 v;
	v.w = *(const f4*)(s.w32 + i);
	v.m1 = *(const f4*)(s.m1 + i);
	v.m2 = *(const f4*)(s.m2 + i);
	v.st = *(const uint4*)(s.steps + i);
	v.w16 = *(const h4*)(s.w16 + i);
	return v;
}

// adam_update on parameters i .. i+3 from their loaded state; same per-parameter arithmetic and
// skip rule. A group with no updated parameter writes nothing back (like the scalar path); otherwise
// skipped parameters are rewritten with their unchanged values.
__device__ __forceinline__ void adam_store4(const AdamArgs& a, const AdamBuffers& s, uint32_t i, const float (&gsum)[4], AdamState4 v) {
	float w[4] = {v.w.x, v.w.y, v.w.z, v.w.w}, m1[4] = {v.m1.x, v.m1.y, v.m1.z, v.m1.w}, m2[4] = {v.m2.x, v.m2.y, v.m2.z, v.m2.w};
	uint32_t st[4] = {v.st.x, v.st.y, v.st.z, v.st.w};
	h4 g16, h = v.w16;
	bool any = false;
#pragma unroll
	for (int r = 0; r < 4; ++r) {
		_Float16 gr;
		const bool upd = adam_core(a, i + r, gsum[r], gr, w[r], m1[r], m2[r], st[r]);
		g16[r] = gr;
		if (upd) h[r] = f16_rn(w[r]);
		any = any || upd;
	}
	if (s.g16) *(h4*)(s.g16 + i) = g16;
	if (!any) return;
	*(f4*)(s.w32 + i) = f4{w[0], w[1], w[2], w[3]};
	*(f4*)(s.m1 + i) = f4{m1[0], m1[1], m1[2], m1[3]};
	*(f4*)(s.m2 + i) = f4{m2[0], m2[1], m2[2], m2[3]};
	*(uint4*)(s.steps + i) = make_uint4(st[0], st[1], st[2], st[3]);
	*(h4*)(s.w16 + i) = h;
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

// Column sums of n_parts fp32 slabs part[j * N + c], columns [c0, c0 + ncol), by ONE workgroup in a
// fixed order (ncol, c0, N multiples of 4): the parts are split into S = blockDim / (ncol / 4)
// contiguous groups; thread (s, k) sums group s of 4-column k (slab_sum order); the S group sums
// are then added in group order. out[c - c0] and tmp (S * ncol floats) are LDS.
__device__ __forceinline__ void block_column_sums(const float* __restrict__ part, uint32_t n_parts, uint32_t N, uint32_t c0, uint32_t ncol,
                                         float* tmp, float* out) {
	const uint32_t nc4 = ncol / 4;
	const uint32_t S = nc4 ? max(1u, blockDim.x / nc4) : 1u;
	const uint32_t per = (n_parts + S - 1) / S;
	const uint32_t t = threadIdx.x;
	if (t < S * nc4) {
		const uint32_t s = t / nc4, k = t % nc4;
		const uint32_t j0 = s * per, j1 = min(n_parts, j0 + per);
		const f4 v = j0 < j1 ? slab_sum((const f4*)(part + (size_t)j0 * N + c0) + k, N / 4, j1 - j0) : f4{0.0f, 0.0f, 0.0f, 0.0f};
		*(f4*)(tmp + s * ncol + 4 * k) = v;
	}
	__syncthreads();
	for (uint32_t c = t; c < ncol; c += blockDim.x) {
		float a = 0.0f;
		for (uint32_t s = 0; s < S; ++s) a += tmp[s * ncol + c];
		out[c] = a;
	}
	__syncthreads();
}

// Columns per workgroup when G workgroups split N columns (multiple of 4).
__host__ __device__ inline uint32_t column_block(uint32_t N, uint32_t G) { return (N / 4 + G - 1) / G * 4; }

// Fixed-order sum of x[0..n) by one workgroup (strided per-thread sums, then a pairwise LDS tree);
// lds: blockDim floats. Result returned to thread 0.
__device__ __forceinline__ float block_sum_fixed(const float* __restrict__ x, uint32_t n, float* lds) {
	float a = 0.0f;
	for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) a += x[i];
	lds[threadIdx.x] = a;
	__syncthreads();
	for (uint32_t h = blockDim.x / 2; h > 0; h >>= 1) {
		if (threadIdx.x < h) lds[threadIdx.x] += lds[threadIdx.x + h];
		__syncthreads();
	}
	return lds[0];
}

}  // namespace tcnn_amd
