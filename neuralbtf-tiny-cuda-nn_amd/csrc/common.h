// common.h -- shared device/host definitions of the MI355X (gfx950) engine.
//
// Written for CDNA4 only: wave64, MFMA f32_16x16x32_f16, packed-fp16 VALU, 160 KiB LDS per CU.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace tcnn_amd {

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef short s4 __attribute__((ext_vector_type(4)));

constexpr int WAVE = 64;
constexpr uint32_t MAX_LEVELS = 64;
constexpr uint32_t BATCH_GRANULARITY = 256;  // BATCH_SIZE_GRANULARITY, reference common.h:235

#define TCNN_HIP_CHECK(x)                                                                          \
	do {                                                                                       \
		hipError_t _e = (x);                                                               \
		if (_e != hipSuccess)                                                              \
			throw std::runtime_error(std::string(#x " failed: ") + hipGetErrorString(_e) + \
			                         " at " __FILE__ ":" + std::to_string(__LINE__));     \
	} while (0)

#define TCNN_CHECK(cond, msg)                                                                      \
	do {                                                                                       \
		if (!(cond)) throw std::runtime_error(std::string(msg));                          \
	} while (0)

// Per-level grid geometry handed to kernels (computed once on the host, so the kernels and the
// offset table use bit-identical scales/resolutions; reference grid.h:694 vs grid.h:97-98).
struct GridLevels {
	uint32_t n_levels;
	uint32_t offset[MAX_LEVELS + 1];  // in entries
	float scale[MAX_LEVELS];
	uint32_t res[MAX_LEVELS];
	uint32_t dense_stride_ok[MAX_LEVELS];  // helper bitfield (unused by kernels)
};

enum class GridType : uint32_t { Hash = 0, Dense = 1, Tiled = 2 };
enum class HashType : uint32_t { Prime = 0, CoherentPrime = 1, ReversedPrime = 2 };
enum class Interp : uint32_t { Nearest = 0, Linear = 1, Smoothstep = 2 };

// Grid options the fused engine does not take (reference grid_interface.h:101-123, grid.h:284-298):
// max_level masking -- a fraction of the levels, scalar or one value per point (levels above
// max_level * n_levels output 0 and receive no gradient) -- and stochastic interpolation (the
// backward sends each point's gradient to one random corner of its cell).
struct GridOpts {
	float max_level = 1000.0f;
	const float* max_level_gpu = nullptr;  // [B] per point, overrides max_level
	uint32_t stochastic = 0;
	uint32_t n_features = 0;  // n_levels * F (num_grid_features)
	uint32_t active = 0;      // any option in effect (uniform fast-path test)
	uint32_t n_levels = 0;    // set by the forward launcher (AoS lane mapping)
	uint32_t inrange_index = 0;  // grid_index_inrange is exact for in-range positions (Linear)
};

struct GridDesc {
	uint32_t n_pos_dims;
	uint32_t n_features_per_level;
	uint32_t n_levels;
	uint32_t log2_hashmap_size;
	uint32_t base_resolution;
	float per_level_scale;
	GridType grid_type;
	HashType hash_type;
	Interp interp;
};

// fp32 -> fp16 of an fp32 RESULT, rounded once from the fp32 value (the reference's __float2half of
// an fp32 expression). The empty asm pins the fp32 value: without it hipcc folds the producing
// multiply / FMA / subtraction and the conversion into one v_fma_mix{lo,hi}_f16, which rounds the
// exact result straight to fp16 -- different from fp32-then-fp16 whenever the fp32 rounding lands
// on an fp16 tie (~1e-5 of the grid's corner weights; found by tests/test_gpu_grid_large.py).
__device__ __forceinline__ _Float16 f16_rn(float x) {
	asm("" : "+v"(x));
	return (_Float16)x;
}

// The torch binding's parameter gradient from the engine's fp32 sum g of loss-scaled gradients:
// fp16(fp16(g) / s) -- the reference's fp16 gradient divided by the loss scale in fp16 arithmetic
// (modules.py:128-138). One definition for k_grad_finalize and the reductions that fold it in.
__device__ __forceinline__ void grad_finalize_store(float g, float s, void* out, size_t i, int out_f32) {
	const _Float16 h = f16_rn((float)(_Float16)g / s);
	if (out_f32) ((float*)out)[i] = (float)h;
	else ((_Float16*)out)[i] = h;
}

// N fp32 values (N even) -> fp16, each rounded once from its fp32 value, as pairs: a two-element
// conversion selects v_cvt_pk_f16_f32, which hipcc does not fold with the producing multiplies into
// a v_fma_mix (a lone scalar conversion of a product it does fold, even under `fp contract(off)`).
// No asm barrier, so the producers stay free to schedule. tests/test_isa_rounding.py pins the result.
template <uint32_t N>
__device__ __forceinline__ void f16_rn_pairs(const float (&x)[N], _Float16 (&h)[N]) {
	static_assert(N % 2 == 0, "pairs");
#pragma unroll
	for (uint32_t c = 0; c < N; c += 2) {
		const h2 p = __builtin_convertvector((f2v){x[c], x[c + 1]}, h2);
		h[c] = p[0];
		h[c + 1] = p[1];
	}
}

// Engine log (reference common_host.h:46-66: LogSeverity, log_callback, log_info/debug/warning).
// Messages go to the callback installed through tcnn_set_log_callback (capi.cpp); without one they
// are dropped (the reference's default prints to stdout; a library embedded in a torch process should
// not). Severity values are the reference's enum order.
enum class LogSeverity : int { Info = 0, Debug = 1, Warning = 2, Error = 3, Success = 4 };
void log_msg(LogSeverity s, const std::string& msg);
inline void log_debug(const std::string& m) { log_msg(LogSeverity::Debug, m); }
inline void log_warning(const std::string& m) { log_msg(LogSeverity::Warning, m); }

inline uint32_t div_round_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device): the attribute is
// per-device state, so one process-wide "done" flag would skip every device after the first.
// done: the caller's static mask, one bit per device ordinal (mod 64; setting it again is harmless).
inline void set_dyn_lds(const void* kernel, int bytes, uint64_t& done) {
	int dev = 0;
	TCNN_HIP_CHECK(hipGetDevice(&dev));
	const uint64_t bit = 1ull << (dev & 63);
	if (__atomic_load_n(&done, __ATOMIC_ACQUIRE) & bit) return;
	TCNN_HIP_CHECK(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
	__atomic_fetch_or(&done, bit, __ATOMIC_RELEASE);
}

// Grow-only scratch allocation owned by a launcher (not stream-ordered: callers on one stream).
struct DevBufLite {
	void* p = nullptr;
	size_t bytes = 0;
	void* get(size_t n) {
		if (n > bytes) {
			if (p) (void)hipFree(p);
			TCNN_HIP_CHECK(hipMalloc(&p, n));
			bytes = n;
		}
		return p;
	}
};

}  // namespace tcnn_amd
