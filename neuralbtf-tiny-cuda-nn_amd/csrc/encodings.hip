// encodings.hip -- OneBlob and Identity encodings for gfx950 (reference encodings/oneblob.h,
// encodings/identity.h). Output AoS fp16 [B][out_stride] (their preferred layout), padding
// columns set to 1 (oneblob.h:200-203, identity.h:62-63).
#include "kernels.h"

namespace tcnn_amd {

// quartic_cdf / quartic (common_device.h:905-920). The reference is compiled by nvcc with FMA
// contraction on; its contraction points are written out as explicit FMAs here (this file is
// compiled with -ffp-contract=off), the same ones the oracle uses.
__device__ __forceinline__ float quartic_cdf(float x, float inv_radius) {
	const float u = x * inv_radius;
	const float u2 = u * u;
	const float u4 = u2 * u2;
	float p = __builtin_fmaf(-(2.0f / 3.0f), u2, 1.0f);
	p = __builtin_fmaf(1.0f / 5.0f, u4, p);
	return fmaxf(0.0f, fminf(1.0f, __builtin_fmaf((15.0f / 16.0f) * u, p, 0.5f)));
}

__device__ __forceinline__ float quartic_cdf_deriv(float x, float inv_radius) {
	const float u = x * inv_radius;
	const float tmp = fmaxf(__builtin_fmaf(-u, u, 1.0f), 0.0f);
	return (15.0f / 16.0f) * tmp * tmp * inv_radius;
}

// Wrapped CDF at a bin's left boundary (one_blob_subwarp_aligned, oneblob.h:48-51). The two wrap
// terms are clamped for all but the bins within one bin width of the domain's ends: quartic_cdf is
// exactly 0 for u <= -T and exactly 1 for u >= T with T = 1.0625 (every fp32 u checked with this op
// sequence by tools/quartic_clamp_check.c; the last unclamped values are at |u| ~ 1.004), so those
// terms are skipped when no lane of the wave needs them, with bit-identical sums (same addition order).
// The forward is VALU-bound (27 polynomial evaluations per 8 bins before); this removes ~2/3 of them.
__device__ __forceinline__ float wrapped_cdf(float boundary, float x, float n_bins) {
	constexpr float T = 1.0625f;
	const float d = boundary - x;
	const float c = quartic_cdf(d, n_bins);
	// the ballot makes the test wave-uniform (a scalar branch, not predication); inside it every lane
	// evaluates the term, which is exact either way
	float lo = 0.0f, hi = 1.0f;
	if (__builtin_amdgcn_ballot_w64(!((d - 1.0f) * n_bins <= -T))) lo = quartic_cdf(d - 1.0f, n_bins);
	if (__builtin_amdgcn_ballot_w64(!((d + 1.0f) * n_bins >= T))) hi = quartic_cdf(d + 1.0f, n_bins);
	return c + lo + hi;
}

// OneBlob forward, one thread per (sample, dim): all n_bins outputs of that dimension.
// The reference evaluates each bin's left CDF in its own lane and takes the right CDF from lane
// (bin + 1) with __shfl_sync(..., bin + 1, n_bins) (oneblob.h:53-62). On its 32-lane warps a shuffle
// width above 32 acts as width 32, so for n_bins > 32 the source lane wraps inside each 32-bin
// group: bin b reads the left CDF of bin (b & ~31) + ((b + 1) & 31), and only the last bin of the
// dimension adds the wrap-around 1. This kernel reproduces exactly that (S = min(n_bins, 32)).
__global__ __launch_bounds__(256) void k_oneblob_fwd(uint32_t B, uint32_t D, uint32_t n_bins, uint32_t log2_bins,
                                                      const float* __restrict__ x, uint32_t x_stride, _Float16* __restrict__ out,
                                                      uint32_t out_stride, uint32_t n_pad) {
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= B * (D + (n_pad ? 1 : 0))) return;
	const uint32_t i = t / (D + (n_pad ? 1 : 0)), d = t % (D + (n_pad ? 1 : 0));
	_Float16* row = out + (size_t)i * out_stride;
	if (d == D) {  // padding columns
		for (uint32_t j = 0; j < n_pad; ++j) row[D * n_bins + j] = (_Float16)1.0f;
		return;
	}
	const float xv = x[(size_t)i * x_stride + d];
	const float nb = (float)n_bins;
	const uint32_t S = n_bins < 32 ? n_bins : 32;
	_Float16* o = row + d * n_bins;
	for (uint32_t g = 0; g < n_bins; g += S) {
		const float first = wrapped_cdf(scalbnf((float)g, -(int)log2_bins), xv, nb);
		float left = first;
		for (uint32_t j = 0; j < S; ++j) {
			const uint32_t b = g + j;
			float right;
			if (j + 1 < S) right = wrapped_cdf(scalbnf((float)(b + 1), -(int)log2_bins), xv, nb);
			else right = first + (b == n_bins - 1 ? 1.0f : 0.0f);
			o[b] = f16_rn(right - left);
			left = right;
		}
	}
}

// Same values, 8 bins per thread and one 16-byte store (n_bins >= 8): consecutive threads write
// consecutive 16 B of a row. Bin b = g + j of the S-bin group g reads cdf(b + 1) for j + 1 < S and
// cdf(g) (+1 for the dimension's last bin) for the group's last bin, exactly as above.
__global__ __launch_bounds__(256) void k_oneblob_fwd8(uint32_t B, uint32_t D, uint32_t n_bins, uint32_t log2_bins,
                                                       const float* __restrict__ x, uint32_t x_stride, _Float16* __restrict__ out,
                                                       uint32_t out_stride) {
	const uint32_t per_row = D * (n_bins / 8);
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= B * per_row) return;
	// n_bins / 8 is a power of two (shifts); so is per_row for D = 1, 2, 4 (no 32-bit udiv sequences)
	const uint32_t lg = log2_bins - 3;
	uint32_t i, rem;
	if ((per_row & (per_row - 1)) == 0) {
		const uint32_t lr = lg + (uint32_t)__builtin_ctz(D);
		i = t >> lr;
		rem = t & (per_row - 1);
	} else {
		i = t / per_row;
		rem = t - i * per_row;
	}
	const uint32_t d = rem >> lg, b0 = 8 * (rem & ((1u << lg) - 1));
	const float xv = x[(size_t)i * x_stride + d];
	const float nb = (float)n_bins;
	const uint32_t S = n_bins < 32 ? n_bins : 32;
	const uint32_t g = b0 & ~(S - 1);
	float left = wrapped_cdf(scalbnf((float)b0, -(int)log2_bins), xv, nb);
	h8 o;
#pragma unroll
	for (uint32_t j = 0; j < 8; ++j) {
		const uint32_t b = b0 + j;
		float right;
		if (b - g + 1 < S) right = wrapped_cdf(scalbnf((float)(b + 1), -(int)log2_bins), xv, nb);
		else right = wrapped_cdf(scalbnf((float)g, -(int)log2_bins), xv, nb) + (b == n_bins - 1 ? 1.0f : 0.0f);
		o[j] = f16_rn(right - left);
		left = right;
	}
	*(h8*)(out + (size_t)i * out_stride + d * n_bins + b0) = o;
}

__global__ __launch_bounds__(256) void k_fill_pad(uint32_t B, _Float16* __restrict__ out, uint32_t out_stride, uint32_t col0,
                                                  uint32_t n_pad) {
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= B * n_pad) return;
	out[(size_t)(t / n_pad) * out_stride + col0 + t % n_pad] = (_Float16)1.0f;
}

// kernel_one_blob_backward (oneblob.h:116-147): dL/dx[d] = sum_k dL/dy[d*n_bins + k] * (D_left - D_right).
__global__ __launch_bounds__(256) void k_oneblob_bwd(uint32_t B, uint32_t D, uint32_t n_bins, uint32_t log2_bins,
                                                      const float* __restrict__ x, uint32_t x_stride,
                                                      const _Float16* __restrict__ dy, uint32_t dy_stride, float* __restrict__ dx,
                                                      uint32_t dx_stride) {
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= B * D) return;
	const uint32_t i = t / D, d = t % D;
	const float xv = x[(size_t)i * x_stride + d];
	const float nb = (float)n_bins;
	float left = quartic_cdf_deriv(-xv, nb) + quartic_cdf_deriv(-xv - 1.0f, nb) + quartic_cdf_deriv(-xv + 1.0f, nb);
	float result = 0.0f;
	for (uint32_t k = 0; k < n_bins; ++k) {
		const float rb = scalbnf((float)(k + 1), -(int)log2_bins);
		const float right = quartic_cdf_deriv(rb - xv, nb) + quartic_cdf_deriv(rb - xv - 1.0f, nb) + quartic_cdf_deriv(rb - xv + 1.0f, nb);
		const float deriv = left - right;
		left = right;
		result = __builtin_fmaf((float)dy[(size_t)i * dy_stride + d * n_bins + k], deriv, result);
	}
	dx[(size_t)i * dx_stride + d] = result;
}

static uint32_t ilog2(uint32_t v) {
	uint32_t r = 0;
	while ((1u << r) < v) ++r;
	return r;
}

void launch_oneblob_fwd(hipStream_t st, uint32_t B, uint32_t D, uint32_t n_bins, const float* x, uint32_t x_stride, void* out16,
                        uint32_t out_stride, uint32_t n_pad) {
	TCNN_CHECK(n_bins > 0 && (n_bins & (n_bins - 1)) == 0, "Number of bins must be a power of 2");
	if (!B) return;
	if (n_bins >= 8 && out_stride % 8 == 0) {
		const uint32_t n = B * D * (n_bins / 8);
		hipLaunchKernelGGL(k_oneblob_fwd8, dim3(div_round_up(n, 256)), dim3(256), 0, st, B, D, n_bins, ilog2(n_bins), x, x_stride,
		                   (_Float16*)out16, out_stride);
		if (n_pad)
			hipLaunchKernelGGL(k_fill_pad, dim3(div_round_up(B * n_pad, 256)), dim3(256), 0, st, B, (_Float16*)out16, out_stride,
			                   D * n_bins, n_pad);
	} else {
		const uint32_t n = B * (D + (n_pad ? 1 : 0));
		hipLaunchKernelGGL(k_oneblob_fwd, dim3(div_round_up(n, 256)), dim3(256), 0, st, B, D, n_bins, ilog2(n_bins), x, x_stride,
		                   (_Float16*)out16, out_stride, n_pad);
	}
	TCNN_HIP_CHECK(hipGetLastError());
}

void launch_oneblob_bwd(hipStream_t st, uint32_t B, uint32_t D, uint32_t n_bins, const float* x, uint32_t x_stride,
                        const void* dy16, uint32_t dy_stride, float* dx, uint32_t dx_stride) {
	if (!B) return;
	hipLaunchKernelGGL(k_oneblob_bwd, dim3(div_round_up(B * D, 256)), dim3(256), 0, st, B, D, n_bins, ilog2(n_bins), x, x_stride,
	                   (const _Float16*)dy16, dy_stride, dx, dx_stride);
	TCNN_HIP_CHECK(hipGetLastError());
}

// identity (identity.h:45-66): out = x * scale + offset (nvcc contracts to one FMA), padding 1.
__global__ __launch_bounds__(256) void k_identity_fwd(uint32_t B, uint32_t D, float scale, float offset, const float* __restrict__ x,
                                                       uint32_t x_stride, _Float16* __restrict__ out, uint32_t out_stride,
                                                       uint32_t n_pad) {
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t fan = D + n_pad;
	if (t >= B * fan) return;
	const uint32_t i = t / fan, j = t % fan;
	out[(size_t)i * out_stride + j] = j < D ? f16_rn(__builtin_fmaf(x[(size_t)i * x_stride + j], scale, offset)) : (_Float16)1.0f;
}

// identity_backward (identity.h:68-85): dL/dx = (T)(dL/dy * scale) -- stored as fp32 here.
__global__ __launch_bounds__(256) void k_identity_bwd(uint32_t B, uint32_t D, float scale, const _Float16* __restrict__ dy,
                                                       uint32_t dy_stride, float* __restrict__ dx, uint32_t dx_stride) {
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= B * D) return;
	const uint32_t i = t / D, j = t % D;
	dx[(size_t)i * dx_stride + j] = (float)f16_rn((float)dy[(size_t)i * dy_stride + j] * scale);
}

void launch_identity_fwd(hipStream_t st, uint32_t B, uint32_t D, float scale, float offset, const float* x, uint32_t x_stride,
                         void* out16, uint32_t out_stride, uint32_t n_pad) {
	if (!B) return;
	hipLaunchKernelGGL(k_identity_fwd, dim3(div_round_up(B * (D + n_pad), 256)), dim3(256), 0, st, B, D, scale, offset, x, x_stride,
	                   (_Float16*)out16, out_stride, n_pad);
	TCNN_HIP_CHECK(hipGetLastError());
}

void launch_identity_bwd(hipStream_t st, uint32_t B, uint32_t D, float scale, const void* dy16, uint32_t dy_stride, float* dx,
                         uint32_t dx_stride) {
	if (!B) return;
	hipLaunchKernelGGL(k_identity_bwd, dim3(div_round_up(B * D, 256)), dim3(256), 0, st, B, D, scale, (const _Float16*)dy16, dy_stride,
	                   dx, dx_stride);
	TCNN_HIP_CHECK(hipGetLastError());
}

}  // namespace tcnn_amd
