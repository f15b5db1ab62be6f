// fused.hip -- gfx950 fused grid-encoding + MLP train step and MLP inference launchers
// (kernels in mlp_fused.h). Split from kernels.hip so the heavy template instantiations compile
// in their own translation unit.
#include "kernels.h"

#include <cstdlib>

#include "grid_device.h"
#include "mlp_fused.h"

namespace tcnn_amd {
// =============================================================================================
// fused train step
// =============================================================================================

// (W64 with 3 hidden layers is not here: its dW accumulators spilled 126-216 registers at 256 and
// it trained 1.45x slower than on the tile engine, profiles/r03_engine_choice_ab.json)
#define TCNN_FUSED_SHAPES(X) \
	X(64, 32, 2)             \
	X(64, 32, 1)             \
	X(32, 32, 2)             \
	X(32, 32, 1)

bool fused_train_supported(uint32_t W, uint32_t IN, uint32_t NH, uint32_t D, uint32_t F, uint32_t OUTP, int act, HashType h) {
	if (F != 2 || OUTP != 16 || (D != 2 && D != 3) || (act != 0 && act != 1)) return false;
#define X(w, in, nh) if (W == w && IN == in && NH == nh) return true;
	TCNN_FUSED_SHAPES(X)
#undef X
	return false;
}

size_t fused_weight_image_bytes(uint32_t W, uint32_t IN, uint32_t NH) {
#define X(w, in, nh) if (W == w && IN == in && NH == nh) return (size_t)FusedLayout<w, in, nh>::oStage * 2;
	TCNN_FUSED_SHAPES(X)
#undef X
	return 0;
}

void launch_pack_weights(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, const void* params16, void* image) {
#define X(w, in, nh)                                                                                               \
	if (W == w && IN == in && NH == nh) {                                                                          \
		hipLaunchKernelGGL((k_pack_weights<w, in, nh>), dim3(8), dim3(256), 0, st, (const _Float16*)params16, (_Float16*)image); \
		TCNN_HIP_CHECK(hipGetLastError());                                                                         \
		return;                                                                                                    \
	}
	TCNN_FUSED_SHAPES(X)
#undef X
	throw std::runtime_error("pack weights: unsupported shape");
}

void fused_image_layout(uint32_t W, uint32_t IN, uint32_t NH, uint32_t* RSI, uint32_t* RSW, uint32_t* oWh, uint32_t* oWo) {
#define X(w, in, nh)                                                                      \
	if (W == w && IN == in && NH == nh) {                                                 \
		using L = FusedLayout<w, in, nh>;                                                 \
		*RSI = L::RSI; *RSW = L::RSW; *oWh = L::oWh; *oWo = L::oWo;                       \
		return;                                                                           \
	}
	TCNN_FUSED_SHAPES(X)
#undef X
	throw std::runtime_error("fused image layout: unsupported shape");
}

static uint32_t device_cu_count() {
	int dev = 0, n = 0;
	TCNN_HIP_CHECK(hipGetDevice(&dev));
	static int cached_dev = -1;
	static uint32_t cached = 0;
	if (dev != cached_dev) {
		TCNN_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
		cached = n > 0 ? (uint32_t)n : 1u;
		cached_dev = dev;
	}
	return cached;
}

uint32_t fused_train_waves() { return FUSED_WAVES; }

uint32_t fused_train_n_blocks(uint32_t W, uint32_t IN, uint32_t NH, uint32_t D, uint32_t dims, bool ext_dout, uint32_t B) {
	const uint32_t n_cu = device_cu_count();
	// FUSED_WAVES waves x 32 samples per workgroup iteration; 8 waves per CU, persistent.
	const uint32_t nb = div_round_up(B, 32u * FUSED_WAVES);
	const uint32_t cap = (8u / FUSED_WAVES) * n_cu;
	return nb < cap ? nb : cap;
}

template <int W, int IN, int NH, uint32_t D, HashType H, Act A, bool EXT, bool ENC = false>
static void launch_fused_e(hipStream_t st, const FusedTrainArgs& args, uint32_t n_blocks) {
	constexpr size_t bytes = RegKernelLayout<W, IN, NH>::BYTES;
	static uint64_t done = 0;
	set_dyn_lds((const void*)k_fused_train_grid<W, IN, NH, D, H, A, EXT, ENC>, (int)bytes, done);
	hipLaunchKernelGGL((k_fused_train_grid<W, IN, NH, D, H, A, EXT, ENC>), dim3(n_blocks), dim3(64 * FUSED_WAVES), bytes, st, args);
	TCNN_HIP_CHECK(hipGetLastError());
}

template <int W, int IN, int NH, uint32_t D, HashType H, Act A>
static void launch_fused_t(hipStream_t st, const FusedTrainArgs& args, uint32_t n_blocks) {
	if (args.enc) {
		// the encoding comes from memory: one instantiation serves every D / hash
		if (args.dout) launch_fused_e<W, IN, NH, 2, HashType::CoherentPrime, A, true, true>(st, args, n_blocks);
		else launch_fused_e<W, IN, NH, 2, HashType::CoherentPrime, A, false, true>(st, args, n_blocks);
	} else if (args.dout) {
		launch_fused_e<W, IN, NH, D, H, A, true>(st, args, n_blocks);
	} else {
		launch_fused_e<W, IN, NH, D, H, A, false>(st, args, n_blocks);
	}
}

template <int W, int IN, int NH>
static void launch_fused_shape(hipStream_t st, uint32_t D, HashType h, int act, const FusedTrainArgs& a, uint32_t nb) {
#define DISPATCH_H(DD, AA)                                                                                   \
	switch (h) {                                                                                          \
		case HashType::Prime: launch_fused_t<W, IN, NH, DD, HashType::Prime, AA>(st, a, nb); break;       \
		case HashType::ReversedPrime: launch_fused_t<W, IN, NH, DD, HashType::ReversedPrime, AA>(st, a, nb); break; \
		default: launch_fused_t<W, IN, NH, DD, HashType::CoherentPrime, AA>(st, a, nb); break;            \
	}
	if (D == 2) {
		if (act == 1) { DISPATCH_H(2, Act::ReLU) } else { DISPATCH_H(2, Act::None) }
	} else {
		if (act == 1) { DISPATCH_H(3, Act::ReLU) } else { DISPATCH_H(3, Act::None) }
	}
#undef DISPATCH_H
}

void launch_fused_train(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, uint32_t D, HashType h, int act,
                        uint32_t B, uint32_t dims, float loss_scale, const void* params16, const void* table16,
                        const float* pos, const float* target, void* out16, void* dLdenc_pairs,
                        float* wgrad_partial, float* loss_partial, const LevelInfo* levels, bool hash_grid,
                        Interp interp, uint32_t n_blocks, const void* dout16, const void* wimage, uint32_t loss_l2,
                        bool inrange_index, const void* enc16, float dout_scale) {
	TCNN_CHECK(B % 32 == 0, "fused train: batch must be a multiple of 32");
	TCNN_CHECK(wimage || ((uintptr_t)params16 & 15) == 0, "fused train: parameters must be 16-byte aligned");
	FusedTrainArgs a;
	a.enc = (const _Float16*)enc16;
	a.loss_l2 = loss_l2;
	a.inrange_index = inrange_index ? 1u : 0u;
	a.wimage = (const _Float16*)wimage;
	a.dout = (const _Float16*)dout16;
	a.dout_scale = dout_scale;
	a.B = B;
	a.dims = dims;
	a.loss_scale = loss_scale;
	a.n_total = (float)(B * dims);
	a.params = (const _Float16*)params16;
	a.table = (const uint32_t*)table16;
	a.pos = pos;
	a.target = target;
	a.out = (_Float16*)out16;
	a.dLdenc = (uint32_t*)dLdenc_pairs;
	a.wgrad_partial = wgrad_partial;
	a.loss_partial = loss_partial;
	a.levels = levels;
	a.hash_grid = hash_grid ? 1u : 0u;
	a.interp = (uint32_t)interp;
	a.prof = nullptr;
#define X(w, in, nh) if (W == w && IN == in && NH == nh) { launch_fused_shape<w, in, nh>(st, D, h, act, a, n_blocks); return; }
	TCNN_FUSED_SHAPES(X)
#undef X
	throw std::runtime_error("fused train: unsupported shape");
}

template <int W, int IN, int NH, Act A, bool SOA>
static void launch_infer_t(hipStream_t st, uint32_t B, const void* wimage, const void* in, void* out) {
	constexpr size_t bytes = (size_t)FusedLayout<W, IN, NH>::oStage * 2;
	static uint64_t done = 0;
	set_dyn_lds((const void*)k_mlp_infer<W, IN, NH, A, SOA>, (int)bytes, done);
	uint32_t nb = div_round_up(B, 64);
	if (nb > 1024) nb = 1024;
	hipLaunchKernelGGL((k_mlp_infer<W, IN, NH, A, SOA>), dim3(nb), dim3(256), bytes, st, B, (const _Float16*)wimage,
	                   (const _Float16*)in, (_Float16*)out);
	TCNN_HIP_CHECK(hipGetLastError());
}

bool mlp_infer_supported(uint32_t W, uint32_t IN, uint32_t NH, uint32_t OUTP, int act) {
	if (OUTP != 16 || (act != 0 && act != 1)) return false;
#define X(w, in, nh) if (W == w && IN == in && NH == nh) return true;
	TCNN_FUSED_SHAPES(X)
#undef X
	return false;
}

void launch_mlp_infer(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, int act, bool soa, uint32_t B,
                      const void* wimage, const void* in16, void* out16) {
	TCNN_CHECK(B % 16 == 0, "mlp inference: batch must be a multiple of 16");
	if (B == 0) return;
#define X(w, in, nh)                                                                                      \
	if (W == w && IN == in && NH == nh) {                                                                 \
		if (act == 1) { if (soa) launch_infer_t<w, in, nh, Act::ReLU, true>(st, B, wimage, in16, out16);   \
		                else launch_infer_t<w, in, nh, Act::ReLU, false>(st, B, wimage, in16, out16); }    \
		else { if (soa) launch_infer_t<w, in, nh, Act::None, true>(st, B, wimage, in16, out16);            \
		       else launch_infer_t<w, in, nh, Act::None, false>(st, B, wimage, in16, out16); }             \
		return;                                                                                           \
	}
	TCNN_FUSED_SHAPES(X)
#undef X
	throw std::runtime_error("mlp inference: unsupported shape");
}

template <int W, int IN, int NH, uint32_t D, HashType H, Act A>
static void launch_fused_fwd_t(hipStream_t st, const FusedFwdArgs& a) {
	constexpr size_t bytes = FwdLayout<W, IN, NH>::BYTES;
	static uint64_t done = 0;
	set_dyn_lds((const void*)k_fused_fwd_grid<W, IN, NH, D, H, A>, (int)bytes, done);
	uint32_t nb = div_round_up(a.B, 16u * FWD_WAVES);
	const uint32_t cap = 3 * device_cu_count();  // 41 KB of LDS per 8-wave workgroup: 3 per CU
	if (nb > cap) nb = cap;
	hipLaunchKernelGGL((k_fused_fwd_grid<W, IN, NH, D, H, A>), dim3(nb), dim3(64 * FWD_WAVES), bytes, st, a);
	TCNN_HIP_CHECK(hipGetLastError());
}

template <int W, int IN, int NH>
static void launch_fused_fwd_shape(hipStream_t st, uint32_t D, HashType h, int act, const FusedFwdArgs& a) {
#define DISPATCH_H(DD, AA)                                                                                   \
	switch (h) {                                                                                          \
		case HashType::Prime: launch_fused_fwd_t<W, IN, NH, DD, HashType::Prime, AA>(st, a); break;       \
		case HashType::ReversedPrime: launch_fused_fwd_t<W, IN, NH, DD, HashType::ReversedPrime, AA>(st, a); break; \
		default: launch_fused_fwd_t<W, IN, NH, DD, HashType::CoherentPrime, AA>(st, a); break;            \
	}
	if (D == 2) {
		if (act == 1) { DISPATCH_H(2, Act::ReLU) } else { DISPATCH_H(2, Act::None) }
	} else {
		if (act == 1) { DISPATCH_H(3, Act::ReLU) } else { DISPATCH_H(3, Act::None) }
	}
#undef DISPATCH_H
}

void launch_fused_fwd(hipStream_t st, uint32_t W, uint32_t IN, uint32_t NH, uint32_t D, HashType h, int act, uint32_t B,
                      const void* wimage, const void* params16, const void* table16, const float* pos, const LevelInfo* levels, bool hash_grid,
                      Interp interp, bool inrange_index, void* enc16, void* out16) {
	TCNN_CHECK(B % 16 == 0, "fused forward: batch must be a multiple of 16");
	if (B == 0) return;
	FusedFwdArgs a;
	a.B = B;
	TCNN_CHECK(wimage || ((uintptr_t)params16 & 15) == 0, "fused forward: parameters must be 16-byte aligned");
	a.wimage = (const _Float16*)wimage;
	a.params = (const _Float16*)params16;
	a.table = (const uint32_t*)table16;
	a.pos = pos;
	a.levels = levels;
	a.hash_grid = hash_grid ? 1u : 0u;
	a.interp = (uint32_t)interp;
	a.inrange_index = inrange_index ? 1u : 0u;
	a.enc = (_Float16*)enc16;
	a.out = (_Float16*)out16;
#define X(w, in, nh) if (W == w && IN == in && NH == nh) { launch_fused_fwd_shape<w, in, nh>(st, D, h, act, a); return; }
	TCNN_FUSED_SHAPES(X)
#undef X
	throw std::runtime_error("fused forward: unsupported shape");
}

__global__ void k_trim_cast(uint32_t B, uint32_t in_stride, uint32_t n_out, const _Float16* __restrict__ in, float* __restrict__ out) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= B * n_out) return;
	const uint32_t b = i / n_out, o = i % n_out;
	out[i] = (float)in[(size_t)b * in_stride + o];
}

void launch_trim_cast(hipStream_t st, uint32_t B, uint32_t in_stride, uint32_t n_out, const void* in16, float* out) {
	if (!B) return;
	hipLaunchKernelGGL(k_trim_cast, dim3(div_round_up((size_t)B * n_out, 256)), dim3(256), 0, st, B, in_stride, n_out, (const _Float16*)in16, out);
	TCNN_HIP_CHECK(hipGetLastError());
}

void launch_fused_train_profile(hipStream_t st, uint32_t B, uint32_t dims, const void* params16, const void* table16,
                                const float* pos, const float* target, void* dLdenc, float* wgrad_partial,
                                float* loss_partial, const LevelInfo* levels, uint32_t n_blocks, const void* wimage,
                                unsigned long long* prof) {
	TCNN_CHECK(dims <= 3, "phase profile: dims <= 3");
	FusedTrainArgs a{};
	a.wimage = (const _Float16*)wimage;
	a.B = B; a.dims = dims; a.loss_scale = 128.0f; a.n_total = (float)(B * dims);
	a.params = (const _Float16*)params16; a.table = (const uint32_t*)table16; a.pos = pos; a.target = target;
	a.out = nullptr; a.dLdenc = (uint32_t*)dLdenc; a.wgrad_partial = wgrad_partial; a.loss_partial = loss_partial;
	a.levels = levels; a.hash_grid = 1; a.interp = (uint32_t)Interp::Linear; a.dout = nullptr; a.dout_scale = 1.0f; a.enc = nullptr; a.prof = prof;
	a.inrange_index = 1;
	using K = RegKernelLayout<64, 32, 2>;
	static uint64_t done = 0;
	set_dyn_lds((const void*)k_fused_train_grid<64, 32, 2, 2, HashType::CoherentPrime, Act::ReLU, false, false, true>, (int)K::BYTES, done);
	hipLaunchKernelGGL((k_fused_train_grid<64, 32, 2, 2, HashType::CoherentPrime, Act::ReLU, false, false, true>), dim3(n_blocks),
	                   dim3(64 * FUSED_WAVES), K::BYTES, st, a);
	TCNN_HIP_CHECK(hipGetLastError());
}

}  // namespace tcnn_amd
