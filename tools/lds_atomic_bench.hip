// Microbenchmark: LDS atomic / store throughput on gfx950 (informs the grid-backward design).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(1024) void k(float* out, int iters, uint32_t mask) {
	extern __shared__ float acc[];
	for (int j = threadIdx.x; j < 16384; j += blockDim.x) acc[j] = 0.f;
	__syncthreads();
	uint32_t x = (blockIdx.x * 1024u + threadIdx.x) * 2654435761u + 12345u;
	for (int it = 0; it < iters; ++it) {
		x = x * 1664525u + 1013904223u;
		uint32_t a = (MODE == 1) ? ((threadIdx.x + it * 64u) & mask) : ((x >> 8) & mask);
		if (MODE == 0 || MODE == 1) atomicAdd(&acc[a], 1.0f);
		if (MODE == 2) acc[a] = (float)it;
		if (MODE == 3) __hip_atomic_fetch_add((uint32_t*)&acc[a], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
		if (MODE == 5) __hip_atomic_fetch_add((unsigned long long*)__builtin_assume_aligned(&acc[a & ~1u], 8), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
		if (MODE == 6) {  // fp32 -> fixed-point i64 conversion + u64 add (grid backward inner op)
			float cv = (float)(x & 0xffff) * 1e-5f;
			long long iv = (long long)(cv * 0x1p40f);
			__hip_atomic_fetch_add((unsigned long long*)__builtin_assume_aligned(&acc[a & ~1u], 8), (unsigned long long)iv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
		}
		if (MODE == 4) {
			h2 v = {(_Float16)1.0f, (_Float16)1.0f};
			__builtin_amdgcn_ds_atomic_fadd_v2f16((__attribute__((address_space(3))) h2*)&acc[a], v);
		}
	}
	__syncthreads();
	out[blockIdx.x * blockDim.x + threadIdx.x] = acc[threadIdx.x];
}

template <int MODE>
void run(const char* name, float* out, uint32_t mask) {
	int iters = 256;
	hipEvent_t e0, e1;
	hipEventCreate(&e0); hipEventCreate(&e1);
	k<MODE><<<512, 1024, 65536>>>(out, iters, mask);
	hipEventRecord(e0);
	k<MODE><<<512, 1024, 65536>>>(out, iters, mask);
	hipEventRecord(e1);
	hipEventSynchronize(e1);
	float ms; hipEventElapsedTime(&ms, e0, e1);
	double ops = 512.0 * 1024 * iters;
	printf("%-28s mask=%6u  %8.3f ms  %8.2f G lane-ops/s  %6.1f cycles/wave-instr/CU (2.4GHz)\n", name, mask, ms, ops / ms / 1e6,
	       (ms * 1e-3 * 2.4e9) / (512.0 * 16 * iters / 256.0));
}

int main() {
	float* out; hipMalloc(&out, 512 * 1024 * 4);
	hipFuncSetAttribute((const void*)k<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
	for (uint32_t mask : {16383u, 511u}) {
		run<0>("ds_add_f32 random", out, mask);
		run<1>("ds_add_f32 lane-linear", out, mask);
		run<2>("ds_write_b32 random", out, mask);
		run<3>("ds_add_u32 random", out, mask);
		run<4>("ds_pk_add_f16 random", out, mask);
		run<5>("ds_add_u64 random", out, mask);
		run<6>("cvt f32->i64 + ds_add_u64", out, mask);
	}
	return 0;
}
