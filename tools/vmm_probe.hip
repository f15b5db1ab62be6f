// Probe of HIP virtual memory management on the box (arena.cpp): which reserve / map / set-access
// combinations succeed.  hipcc --offload-arch=gfx950 vmm_probe.hip -o vmm_probe
#include <hip/hip_runtime.h>
#include <cstdio>
static void run(size_t reserve, size_t align, int per_chunk_access) {
	int dev = 0;
	hipMemAllocationProp prop = {};
	prop.type = hipMemAllocationTypePinned;
	prop.location.type = hipMemLocationTypeDevice;
	prop.location.id = dev;
	size_t gran = 0;
	hipError_t e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum);
	void* base = nullptr;
	hipError_t r = hipMemAddressReserve(&base, reserve, align, nullptr, 0);
	std::printf("reserve %zu align %zu: gran %zu (%d) reserve=%d base=%p\n", reserve, align, gran, (int)e, (int)r, base);
	if (r != hipSuccess) return;
	size_t off = 0;
	for (int k = 0; k < 2; ++k) {
		hipMemGenericAllocationHandle_t h;
		hipError_t c = hipMemCreate(&h, gran, &prop, 0);
		hipError_t m = hipMemMap((char*)base + off, gran, 0, h, 0);
		hipMemAccessDesc acc = {};
		acc.location.type = hipMemLocationTypeDevice;
		acc.location.id = dev;
		acc.flags = hipMemAccessFlagsProtReadWrite;
		hipError_t a = per_chunk_access ? hipMemSetAccess((char*)base + off, gran, &acc, 1) : hipMemSetAccess(base, off + gran, &acc, 1);
		hipError_t s = hipMemsetD8((hipDeviceptr_t)((char*)base + off), 1, gran);
		std::printf("  chunk %d: create=%d map=%d access=%d memset=%d\n", k, (int)c, (int)m, (int)a, (int)s);
		off += gran;
	}
	hipGetLastError();
}
// a small chunk then a 3 GiB chunk behind it, at 4 KiB and at 2 MiB offsets
static void run_big() {
	hipMemAllocationProp prop = {};
	prop.type = hipMemAllocationTypePinned;
	prop.location.type = hipMemLocationTypeDevice;
	prop.location.id = 0;
	hipMemAccessDesc acc = {};
	acc.location.type = hipMemLocationTypeDevice;
	acc.location.id = 0;
	acc.flags = hipMemAccessFlagsProtReadWrite;
	for (size_t first : {(size_t)4096, (size_t)2 << 20}) {
		void* base = nullptr;
		hipMemAddressReserve(&base, (size_t)64 << 30, 0, nullptr, 0);
		hipMemGenericAllocationHandle_t h0, h1;
		hipMemCreate(&h0, first, &prop, 0);
		hipMemMap(base, first, 0, h0, 0);
		hipError_t a0 = hipMemSetAccess(base, first, &acc, 1);
		const size_t big = (size_t)3 << 30;
		hipError_t c = hipMemCreate(&h1, big, &prop, 0);
		hipError_t m = hipMemMap((char*)base + first, big, 0, h1, 0);
		hipError_t a1 = hipMemSetAccess((char*)base + first, big, &acc, 1);
		hipError_t s = hipMemsetD8((hipDeviceptr_t)((char*)base + first), 1, big);
		std::printf("big after %zu: access0=%d create=%d map=%d access=%d memset=%d\n", first, (int)a0, (int)c, (int)m, (int)a1, (int)s);
		hipGetLastError();
	}
}
int main() {
	size_t fr = 0, tot = 0;
	hipMemGetInfo(&fr, &tot);
	int vm = 0;
	hipDeviceGetAttribute(&vm, hipDeviceAttributeVirtualMemoryManagementSupported, 0);
	std::printf("vmm attr %d total %zu\n", vm, tot);
	run((size_t)1 << 30, 0, 1);
	run((size_t)64 << 30, 0, 1);
	run(tot / ((size_t)2 << 20) * ((size_t)2 << 20), 0, 1);
	run((size_t)64 << 30, 0, 0);
	run_big();
	return 0;
}
