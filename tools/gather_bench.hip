// Gather microbenchmark: does the gfx950 vector L1 (TCP) coalesce lanes of one load instruction that
// hit the same cache line? The fused kernel's grid encode is bound by L1 tag work
// (TA_ADDR_STALLED_BY_TC); if two lanes reading x-neighbour table entries in one instruction cost
// one tag lookup instead of two, a lane-pair gather layout halves that work.
//
// Every lane issues G 4-byte gathers from a 2 MiB table (L2-resident, like config_hash's 16 levels).
// mode 0: every lane a random entry (64 distinct lines per instruction)
// mode 1: lane pairs (2k, 2k+1) read entries e, e^1 (32 distinct lines per instruction)
// mode 2: lane quads read e, e^1, e^2, e^3 (16 lines)
// mode 3: lanes L and L^16 share a line (32 lines, partners 16 lanes apart)
// mode 4: mode 0 with half the gathers (the instruction count of a paired layout)
// Build: hipcc --offload-arch=gfx950 -O3 tools/gather_bench.hip -o tools/gather_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
	do {                                                                           \
		hipError_t e = (x);                                                        \
		if (e != hipSuccess) {                                                     \
			std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
			std::exit(1);                                                          \
		}                                                                          \
	} while (0)

constexpr int G = 32;                  // gathers per lane per iteration
constexpr uint32_t TABLE = 1u << 19;   // entries (2 MiB)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
	x ^= x >> 16;
	x *= 0x7feb352dU;
	x ^= x >> 15;
	x *= 0x846ca68bU;
	x ^= x >> 16;
	return x;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_gather(const uint32_t* __restrict__ table, uint32_t* __restrict__ out, int iters) {
	const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t lane = threadIdx.x & 63;
	uint32_t acc = 0;
	for (int it = 0; it < iters; ++it) {
		uint32_t v[G];
#pragma unroll
		for (int g = 0; g < G; ++g) {
			if (MODE == 4 && g >= G / 2) break;
			uint32_t key;
			if (MODE == 0 || MODE == 4) key = tid;
			else if (MODE == 1) key = tid >> 1;
			else if (MODE == 2) key = tid >> 2;
			else key = (tid & ~63u) | (lane & 15u) | ((lane & 32u) >> 1);  // lanes L, L^16 share a key
			uint32_t e = hash32(key * 977u + (uint32_t)(it * G + g) * 0x9e3779b9u) & (TABLE - 1);
			if (MODE == 1) e ^= lane & 1u;
			else if (MODE == 2) e ^= lane & 3u;
			else if (MODE == 3) e ^= (lane >> 4) & 1u;
			v[g] = table[e];
		}
#pragma unroll
		for (int g = 0; g < G; ++g) {
			if (MODE == 4 && g >= G / 2) break;
			acc += v[g];
		}
	}
	out[tid] = acc;
}

template <int MODE>
static float run(const uint32_t* table, uint32_t* out, int blocks, int iters) {
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	hipLaunchKernelGGL(k_gather<MODE>, dim3(blocks), dim3(256), 0, nullptr, table, out, iters);  // warm-up
	CHECK(hipEventRecord(a));
	for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_gather<MODE>, dim3(blocks), dim3(256), 0, nullptr, table, out, iters);
	CHECK(hipEventRecord(b));
	CHECK(hipEventSynchronize(b));
	float ms = 0;
	CHECK(hipEventElapsedTime(&ms, a, b));
	CHECK(hipEventDestroy(a));
	CHECK(hipEventDestroy(b));
	return ms / 5;
}

int main() {
	int dev = 0, n_cu = 0;
	CHECK(hipGetDevice(&dev));
	CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
	const int blocks = n_cu * 8, iters = 64;  // 8 workgroups of 4 waves per CU
	uint32_t *table, *out;
	CHECK(hipMalloc(&table, TABLE * 4));
	CHECK(hipMalloc(&out, (size_t)blocks * 256 * 4));
	std::vector<uint32_t> h(TABLE);
	for (uint32_t i = 0; i < TABLE; ++i) h[i] = i * 2654435761u;
	CHECK(hipMemcpy(table, h.data(), TABLE * 4, hipMemcpyHostToDevice));
	const double lane_loads = (double)blocks * 256 * iters * G;
	const float t0 = run<0>(table, out, blocks, iters);
	const float t1 = run<1>(table, out, blocks, iters);
	const float t2 = run<2>(table, out, blocks, iters);
	const float t3 = run<3>(table, out, blocks, iters);
	const float t4 = run<4>(table, out, blocks, iters);
	std::printf("{\"cus\": %d, \"lane_gathers\": %.0f,\n", n_cu, lane_loads);
	std::printf(" \"random_64_lines_per_instr_ms\": %.4f, \"ns_per_wave_instr\": %.3f,\n", t0, t0 * 1e6 / (lane_loads / 64));
	std::printf(" \"pairs_L_Lxor1_ms\": %.4f, \"quads_ms\": %.4f, \"pairs_L_Lxor16_ms\": %.4f, \"random_half_instr_ms\": %.4f}\n", t1, t2, t3,
	            t4);
	CHECK(hipFree(table));
	CHECK(hipFree(out));
	return 0;
}
