// Negative control for tools/hazard_scan.py (tests/test_isa_hazards.py): two kernels that each carry
// one MFMA data hazard an inline-asm statement creates and hipcc does not pad. Compiled, never run.
#include <hip/hip_runtime.h>
#include <cstdint>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
// R1: an asm VALU instruction reads the MFMA accumulator directly (round 3's bug)
__global__ void r1(const h8* a, const h8* b, uint32_t* o) {
	const int i = threadIdx.x;
	const f4 c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[i], (f4){0, 0, 0, 0}, 0, 0, 0);
	uint32_t r;
	asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(c[0]));
	o[i] = r;
}
// R2: an asm VALU instruction writes an MFMA B operand one wait state before the MFMA
__global__ void r2(const h8* a, const u4* b, f4* o) {
	const int i = threadIdx.x;
	u4 v = b[i];
	asm("v_pk_max_f16 %0, 0, %0" : "+v"(v[3]));
	o[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], __builtin_bit_cast(h8, v), (f4){0, 0, 0, 0}, 0, 0, 0);
}
