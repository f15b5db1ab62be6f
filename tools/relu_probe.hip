// Probe of v_pk_max_f16 0, x on gfx950 for the fp16 ReLU (mlp_fused.h act_fwd): prints the result
// bits for -0, +0, tiny negatives, NaNs and infinities.  hipcc --offload-arch=gfx950 -O2 relu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const uint32_t* in, uint32_t* out, int n) {
	int i = threadIdx.x;
	if (i < n) {
		uint32_t r;
		asm volatile("v_pk_max_f16 %0, 0, %1" : "=v"(r) : "v"(in[i]));
		out[i] = r;
	}
}
int main() {
	const uint32_t v[] = {0x80000000u, 0x00008000u, 0x80008000u, 0x00000000u, 0x7e00fe00u, 0x7c00fc00u, 0x80013c00u, 0xbc000001u, 0x7fff8001u};
	const int n = sizeof(v) / 4;
	uint32_t *di, *dout, h[16];
	hipMalloc(&di, 64); hipMalloc(&dout, 64);
	hipMemcpy(di, v, sizeof(v), hipMemcpyHostToDevice);
	hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, di, dout, n);
	hipMemcpy(h, dout, sizeof(v), hipMemcpyDeviceToHost);
	for (int i = 0; i < n; ++i) printf("in %08x -> %08x\n", v[i], h[i]);
	return 0;
}
