// lds_dma.h -- one dword per lane from global memory into LDS at l + 4 lane (global_load_lds_dword),
// as inline asm. Not __builtin_amdgcn_global_load_lds: with the builtin the compiler cannot tell the
// staging buffers from the rest of the one dynamic LDS array and puts a vmcnt(0) before every later
// LDS read and barrier (mlp_tile.h GENC, measured +30 %). The waits are the caller's: each wave reads
// back only what it loaded itself, after its own s_waitcnt vmcnt. (The compiler then counts fewer
// outstanding vector-memory operations than there are, which only makes its own waits stricter.)
// M0 (the destination base) is reserved by the compiler: saved and restored inside the statement,
// with the wait state an SALU write of M0 needs before the LDS-DMA reads it.
#pragma once
#include <cstdint>

namespace tcnn_amd {

__device__ __forceinline__ uint32_t lds_addr(const void* l) {
	return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)l;
}

// 64-bit per-lane source address
__device__ __forceinline__ void lds_dma_u32(const void* g, const void* l) {
	uint32_t keep;
	asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
	             : "=&s"(keep)
	             : "v"(g), "s"(lds_addr(l))
	             : "memory");
}

// scalar base + 32-bit per-lane byte offset (the saddr form: one VGPR per address, not two)
__device__ __forceinline__ void lds_dma_u32(const void* sbase, uint32_t voff, const void* l) {
	uint32_t keep;
	asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
	             : "=&s"(keep)
	             : "v"(voff), "s"(sbase), "s"(lds_addr(l))
	             : "memory");
}

}  // namespace tcnn_amd
