// grid_bin.hip -- binned grid backward for levels whose gradient accumulators do not fit the LDS
// (reference kernel_grid_backward, grid.h:214-320, launched grid.h:857-880).
//
// The reference scatters every (point, level, corner) update into the gradient table with fp16
// half2 atomics (grid.h:252-255). On gfx950 a global atomic to a random line costs ~17x a coalesced
// one (MI355X_MICROARCH.md, global float atomics), and a 2^19-entry level does not fit a CU's LDS,
// so the large levels go through two passes instead:
//   k_grid_bin  one workgroup per (level, chunk of points): computes the level's corners, ranks each
//               update inside its slice (LDS counters with return), and writes the chunk's updates as
//               records sorted by slice -- one contiguous run per slice -- plus a directory entry
//               {first record, count} per slice and the chunk's sum of |dL/dy|.
//   k_grid_acc  one workgroup per slice: walks the slice's runs of every chunk, adds each update into
//               int32 fixed-point accumulators in LDS, then writes the fp32 gradient of the slice (or
//               applies Adam to those parameters directly). Every table entry belongs to exactly one
//               slice, so there is no cross-workgroup reduction and no partial slab.
// Record: x = (fp16 corner weight << 16) | entry within the slice; y = the point's dL/dy (F <= 2,
// fp16 bits) or its index (F > 2: the accumulator re-reads dL/dy). The product w * dL/dy of two fp16
// values is exact in fp32; its fixed-point image rounds once. Integer sums do not depend on the order
// the records arrive in, so the gradient is bit-reproducible run to run.
// Fixed-point range: an entry of level l receives at most sum_i |dL/dy_i| (the corner weights of a
// point sum to 1, hash collisions included), so scale 2^e with 2^e * (sum + rounding) < 2^31 cannot
// overflow; two's-complement sums are exact modulo 2^32 anyway, so only the final value must fit.
#include "kernels.h"

#include <cstdio>

#include "adam_device.h"
#include "grid_device.h"

namespace tcnn_amd {

constexpr uint32_t BIN_THREADS = 256;
constexpr uint32_t ACC_THREADS = 256;
constexpr uint32_t ACC_DIR_BLOCK = 256;  // chunks whose directory entries sit in LDS at once

// block-wide exclusive scan of v (one value per thread, BIN_THREADS threads); returns the prefix,
// *total gets the sum. scratch: BIN_THREADS / 64 uint32 in LDS.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* scratch, uint32_t* total) {
	const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
	uint32_t x = v;
#pragma unroll
	for (uint32_t o = 1; o < 64; o <<= 1) {
		const uint32_t y = __shfl_up(x, o);
		if (lane >= o) x += y;
	}
	if (lane == 63) scratch[w] = x;
	__syncthreads();
	uint32_t base = 0, tot = 0;
	for (uint32_t j = 0; j < blockDim.x / 64; ++j) {
		const uint32_t s = scratch[j];
		if (j < w) base += s;
		tot += s;
	}
	__syncthreads();
	*total = tot;
	return base + x - v;
}

template <uint32_t D, uint32_t F, HashType H, bool OPTS>
__global__ __launch_bounds__(BIN_THREADS) void k_grid_bin(int layout, uint32_t B, const float* __restrict__ pos, uint32_t pstride,
                                                          const _Float16* __restrict__ dLdy, uint32_t dy_stride,
                                                          const LevelInfo* __restrict__ levels, uint32_t hash_grid, uint32_t interp_u,
                                                          const GridBinArgs a, const GridOpts o) {
	constexpr uint32_t NC = 1u << D;
	constexpr uint32_t PPT = GRID_BIN_RECS / NC / BIN_THREADS;  // points per thread
	static_assert(PPT >= 1, "GRID_BIN_RECS too small for D");
	__shared__ uint2 stage[GRID_BIN_RECS];
	__shared__ uint32_t cnt[GRID_BIN_MAX_SLICES];
	__shared__ uint32_t scratch[BIN_THREADS / 64 * (F > 2 ? F : 2)];
	__shared__ float fsum[BIN_THREADS / 64][F];

	const uint32_t slot = blockIdx.x % a.n_slots, chunk = blockIdx.x / a.n_slots;
	const GridBinLevel bl = a.lv[slot];
	const LevelInfo li = levels[bl.level];
	const Interp interp = (Interp)interp_u;
	const uint32_t n_sl = bl.n_slices;
	const uint32_t smask = (1u << bl.slice_log2) - 1u;
	for (uint32_t s = threadIdx.x; s < n_sl; s += BIN_THREADS) cnt[s] = 0;
	__syncthreads();

	const bool nearest = interp == Interp::Nearest;
	const bool single = nearest || (OPTS && o.stochastic);
	uint32_t rx[PPT][NC], key[PPT][NC], ry[PPT];
	float as[F];
#pragma unroll
	for (uint32_t f = 0; f < F; ++f) as[f] = 0.0f;
#pragma unroll
	for (uint32_t u = 0; u < PPT; ++u) {
		const uint32_t i = chunk * a.pts_per_chunk + u * BIN_THREADS + threadIdx.x;
		bool valid = i < B;
		float x[D], dy[F];
		if (valid) {
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) x[d] = pos[(size_t)i * pstride + d];
			load_dy<F>(layout, dLdy, dy_stride, bl.level, B, i, dy);
			if (OPTS && (float)bl.level > grid_max_level(o, i, F) + 1e-3f) valid = false;  // masked (grid.h:242-244)
		}
		if (!valid) {
#pragma unroll
			for (uint32_t c = 0; c < NC; ++c) key[u][c] = 0xffffffffu;
			ry[u] = 0;
			continue;
		}
		if constexpr (F == 1) {
			ry[u] = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)dy[0]);
		} else if constexpr (F == 2) {
			ry[u] = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)dy[0]) | ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)dy[1]) << 16);
		} else {
			ry[u] = i;
		}
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) as[f] += fabsf(dy[f]);
		float p[D];
		uint32_t pg[D];
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) pos_fract(x[d], li.scale, interp, p[d], pg[d]);
		uint32_t cbits = 0;
		if (single && !nearest) {  // stochastic interpolation (grid.h:284-298)
			const float smp = random_val_1337(i + bl.level * B);
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) cbits |= (smp >= p[d] ? 0u : 1u) << d;
		}
#pragma unroll
		for (uint32_t c0 = 0; c0 < NC; ++c0) {
			if (single && c0 > 0) {
				key[u][c0] = 0xffffffffu;
				continue;
			}
			const uint32_t c = single ? cbits : c0;
			float w = 1.0f;
			uint32_t local[D];
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) {
				if ((c & (1u << d)) == 0) { w *= 1.0f - p[d]; local[d] = pg[d]; }
				else { w *= p[d]; local[d] = pg[d] + 1; }
			}
			const _Float16 wh = single ? (_Float16)1.0f : f16_rn(w);
			const uint32_t idx = grid_index<D, H>(hash_grid != 0, li.size, li.res, local);
			const uint32_t s = idx >> bl.slice_log2;
			const uint32_t rank = atomicAdd(&cnt[s], 1u);
			key[u][c0] = (s << 12) | rank;  // rank < GRID_BIN_RECS = 2^12
			rx[u][c0] = ((uint32_t)__builtin_bit_cast(uint16_t, wh) << 16) | (idx & smask);
		}
	}
	__syncthreads();

	// exclusive scan of the slice counts (each thread owns a contiguous group of slices)
	const uint32_t per = (n_sl + BIN_THREADS - 1) / BIN_THREADS;
	const uint32_t s0 = min(n_sl, threadIdx.x * per), s1 = min(n_sl, s0 + per);
	uint32_t mine = 0;
	for (uint32_t s = s0; s < s1; ++s) mine += cnt[s];
	uint32_t total;
	uint32_t run = block_exclusive_scan(mine, scratch, &total);
	for (uint32_t s = s0; s < s1; ++s) {
		const uint32_t c = cnt[s];
		a.dir[(size_t)(bl.bucket_base + s) * a.n_chunks + chunk] = make_uint2(run, c);
		cnt[s] = run;  // now the slice's first record
		run += c;
	}
	__syncthreads();
#pragma unroll
	for (uint32_t u = 0; u < PPT; ++u)
#pragma unroll
		for (uint32_t c = 0; c < NC; ++c) {
			const uint32_t k = key[u][c];
			if (k != 0xffffffffu) stage[cnt[k >> 12] + (k & 4095u)] = make_uint2(rx[u][c], ry[u]);
		}
	__syncthreads();
	uint4* dst = (uint4*)(a.recs + ((size_t)slot * a.n_chunks + chunk) * GRID_BIN_RECS);
	const uint4* srcv = (const uint4*)stage;
	for (uint32_t j = threadIdx.x; j < (total + 1) / 2; j += BIN_THREADS) dst[j] = srcv[j];

	// chunk sum of |dL/dy| per feature, fixed order (wave tree, then waves in order)
#pragma unroll
	for (uint32_t f = 0; f < F; ++f) {
		float v = as[f];
#pragma unroll
		for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
		if ((threadIdx.x & 63) == 0) fsum[threadIdx.x >> 6][f] = v;
	}
	__syncthreads();
	if (threadIdx.x < F) {
		float v = 0.0f;
		for (uint32_t w = 0; w < BIN_THREADS / 64; ++w) v += fsum[w][threadIdx.x];
		a.dysum[((size_t)slot * a.n_chunks + chunk) * F + threadIdx.x] = v;
	}
}

// fp32 value of a record's update for feature f (exact product of two fp16 values)
template <uint32_t F>
__device__ __forceinline__ void record_values(uint2 r, int layout, const _Float16* __restrict__ dLdy, uint32_t dy_stride, uint32_t level,
                                              uint32_t B, float* v) {
	const float w = (float)__builtin_bit_cast(_Float16, (uint16_t)(r.x >> 16));
	if constexpr (F <= 2) {
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) v[f] = w * (float)__builtin_bit_cast(_Float16, (uint16_t)(r.y >> (16 * f)));
	} else {
		float dy[F];
		load_dy<F>(layout, dLdy, dy_stride, level, B, r.y, dy);
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) v[f] = w * dy[f];
	}
}

template <uint32_t NC, uint32_t F>
__global__ __launch_bounds__(ACC_THREADS) void k_grid_acc(int layout, uint32_t B, const _Float16* __restrict__ dLdy, uint32_t dy_stride,
                                                          const LevelInfo* __restrict__ levels, const GridBinArgs a,
                                                          float* __restrict__ grad32, const GridAccAdam ad, int apply_adam) {
	extern __shared__ __attribute__((aligned(16))) int acc[];
	__shared__ uint32_t pre[ACC_DIR_BLOCK + 1], first[ACC_DIR_BLOCK];
	__shared__ uint32_t scratch[ACC_THREADS / 64];
	__shared__ float fred[ACC_THREADS / 64][F];

	const uint32_t bucket = blockIdx.x;
	uint32_t slot = 0;
	while (slot + 1 < a.n_slots && a.lv[slot + 1].bucket_base <= bucket) ++slot;
	const GridBinLevel bl = a.lv[slot];
	const LevelInfo li = levels[bl.level];
	const uint32_t e0 = (bucket - bl.bucket_base) << bl.slice_log2;
	const uint32_t ne = min(1u << bl.slice_log2, li.size - e0);
	for (uint32_t j = threadIdx.x; j < ne * F; j += ACC_THREADS) acc[j] = 0;

	// fixed-point scale from the level's sum of |dL/dy| (same fixed-order sum in every workgroup of the level)
	float t[F];
#pragma unroll
	for (uint32_t f = 0; f < F; ++f) t[f] = 0.0f;
	for (uint32_t c = threadIdx.x; c < a.n_chunks; c += ACC_THREADS)
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) t[f] += a.dysum[((size_t)slot * a.n_chunks + c) * F + f];
#pragma unroll
	for (uint32_t f = 0; f < F; ++f) {
		float v = t[f];
#pragma unroll
		for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
		if ((threadIdx.x & 63) == 0) fred[threadIdx.x >> 6][f] = v;
	}
	__syncthreads();
	float tmax = 0.0f;
	bool finite = true;
#pragma unroll
	for (uint32_t f = 0; f < F; ++f) {
		float v = 0.0f;
		for (uint32_t w = 0; w < ACC_THREADS / 64; ++w) v += fred[w][f];
		finite = finite && __builtin_isfinite(v);
		tmax = fmaxf(tmax, v);
	}
	int e = 0;
	if (tmax > 0.0f && finite) {
		const float lim = (2147483647.0f - (float)NC * (float)B) / (tmax * 1.01f);
		e = max(-126, min(ilogbf(lim), 100));
	}
	const float scale = ldexpf(1.0f, e);

	// the slice's records, chunk by chunk in blocks of ACC_DIR_BLOCK directory entries, flattened
	for (uint32_t cb = 0; cb < a.n_chunks; cb += ACC_DIR_BLOCK) {
		const uint32_t nb = min(ACC_DIR_BLOCK, a.n_chunks - cb);
		uint2 dv = make_uint2(0, 0);
		if (threadIdx.x < nb) dv = a.dir[(size_t)bucket * a.n_chunks + cb + threadIdx.x];
		uint32_t total;
		const uint32_t ex = block_exclusive_scan(dv.y, scratch, &total);
		if (threadIdx.x < nb) {
			pre[threadIdx.x] = ex;
			first[threadIdx.x] = dv.x;
		}
		if (threadIdx.x == 0) pre[nb] = total;
		__syncthreads();
		constexpr uint32_t U = 8;
		uint32_t c = 0;
		for (uint32_t k0 = threadIdx.x; k0 < total; k0 += U * ACC_THREADS) {
			uint2 r[U];
#pragma unroll
			for (uint32_t u = 0; u < U; ++u) {
				const uint32_t k = k0 + u * ACC_THREADS;
				if (k < total) {
					while (pre[c + 1] <= k) ++c;
					r[u] = a.recs[((size_t)slot * a.n_chunks + cb + c) * GRID_BIN_RECS + first[c] + (k - pre[c])];
				}
			}
#pragma unroll
			for (uint32_t u = 0; u < U; ++u) {
				if (k0 + u * ACC_THREADS >= total) break;
				float v[F];
				record_values<F>(r[u], layout, dLdy, dy_stride, bl.level, B, v);
				const uint32_t loc = r[u].x & 0xffffu;
				if constexpr (F == 2) {
					const int lo = __float2int_rn(v[0] * scale), hi = __float2int_rn(v[1] * scale);
					const unsigned long long pk = (unsigned long long)(((long long)hi << 32) + (long long)lo);
					__hip_atomic_fetch_add((unsigned long long*)acc + loc, pk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
				} else {
#pragma unroll
					for (uint32_t f = 0; f < F; ++f)
						__hip_atomic_fetch_add(acc + loc * F + f, __float2int_rn(v[f] * scale), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
				}
			}
		}
		__syncthreads();
	}

	// write out: grid parameter p = (offset + e0 + entry) * F + f
	const float inv = finite ? ldexpf(1.0f, -e) : __builtin_nanf("");
	const uint32_t p0 = (li.offset + e0) * F;
	auto grad_of = [&](uint32_t j) -> float {
		if constexpr (F == 2) {
			const long long t64 = ((const long long*)acc)[j >> 1];
			const int lo = (int)(uint32_t)(unsigned long long)t64;
			const int hi = (int)((t64 - (long long)lo) >> 32);
			return (float)((j & 1) ? hi : lo) * inv;
		} else {
			return (float)acc[j] * inv;
		}
	};
	if (!apply_adam) {
		for (uint32_t j = threadIdx.x; j < ne * F; j += ACC_THREADS) grad32[p0 + j] = grad_of(j);
		return;
	}
	// Adam on groups of 4 parameters (ne * F and the parameter base are multiples of 4: level offsets
	// are multiples of 8 entries, the network block of 16); two groups per thread have their state
	// loads in flight together
	const uint32_t n4 = ne * F / 4;
	for (uint32_t q0 = threadIdx.x; q0 < n4; q0 += 2 * ACC_THREADS) {
		AdamState4 sv[2];
		float g[2][4];
#pragma unroll
		for (uint32_t u = 0; u < 2; ++u) {
			const uint32_t q = q0 + u * ACC_THREADS;
			if (q < n4) {
				sv[u] = adam_load4(ad.buf, ad.param_base + p0 + 4 * q);
#pragma unroll
				for (uint32_t r = 0; r < 4; ++r) g[u][r] = grad_of(4 * q + r);
			}
		}
#pragma unroll
		for (uint32_t u = 0; u < 2; ++u) {
			const uint32_t q = q0 + u * ACC_THREADS;
			if (q >= n4) break;
			const uint32_t i = ad.param_base + p0 + 4 * q;
			if (ad.write_grad32) *(f4*)(ad.buf.g32 + i) = f4{g[u][0], g[u][1], g[u][2], g[u][3]};
			adam_store4(ad.a, ad.buf, i, g[u], sv[u]);
		}
	}
}

template <uint32_t D, uint32_t F, HashType H>
static void grid_bin_t(hipStream_t st, int layout, uint32_t dys, uint32_t B, const float* pos, uint32_t ps, const _Float16* dy,
                       const LevelInfo* lv, uint32_t hg, uint32_t in, const GridBinArgs& a, const GridOpts& go) {
	const dim3 g(a.n_slots * a.n_chunks);
	if (go.active)
		hipLaunchKernelGGL((k_grid_bin<D, F, H, true>), g, dim3(BIN_THREADS), 0, st, layout, B, pos, ps, dy, dys, lv, hg, in, a, go);
	else
		hipLaunchKernelGGL((k_grid_bin<D, F, H, false>), g, dim3(BIN_THREADS), 0, st, layout, B, pos, ps, dy, dys, lv, hg, in, a, go);
}

template <uint32_t D, uint32_t F>
static void grid_bin_h(hipStream_t st, HashType h, int layout, uint32_t dys, uint32_t B, const float* pos, uint32_t ps, const _Float16* dy,
                       const LevelInfo* lv, uint32_t hg, uint32_t in, const GridBinArgs& a, const GridOpts& go) {
	switch (h) {
		case HashType::Prime: grid_bin_t<D, F, HashType::Prime>(st, layout, dys, B, pos, ps, dy, lv, hg, in, a, go); break;
		case HashType::ReversedPrime: grid_bin_t<D, F, HashType::ReversedPrime>(st, layout, dys, B, pos, ps, dy, lv, hg, in, a, go); break;
		default: grid_bin_t<D, F, HashType::CoherentPrime>(st, layout, dys, B, pos, ps, dy, lv, hg, in, a, go); break;
	}
}

template <uint32_t D>
static void grid_bin_f(hipStream_t st, uint32_t F, HashType h, int layout, uint32_t dys, uint32_t B, const float* pos, uint32_t ps,
                       const _Float16* dy, const LevelInfo* lv, uint32_t hg, uint32_t in, const GridBinArgs& a, const GridOpts& go) {
	switch (F) {
		case 1: grid_bin_h<D, 1>(st, h, layout, dys, B, pos, ps, dy, lv, hg, in, a, go); break;
		case 2: grid_bin_h<D, 2>(st, h, layout, dys, B, pos, ps, dy, lv, hg, in, a, go); break;
		case 4: grid_bin_h<D, 4>(st, h, layout, dys, B, pos, ps, dy, lv, hg, in, a, go); break;
		case 8: grid_bin_h<D, 8>(st, h, layout, dys, B, pos, ps, dy, lv, hg, in, a, go); break;
		default: throw std::runtime_error("GridEncoding: n_features_per_level must be 1, 2, 4 or 8");
	}
}

void launch_grid_bin(hipStream_t st, uint32_t D, uint32_t F, HashType h, uint32_t B, const float* pos, uint32_t pos_stride,
                     const void* dLdy16, int dy_layout, uint32_t dy_stride, const LevelInfo* levels, bool hash_grid, Interp interp,
                     const GridBinArgs& a, const GridOpts& go) {
	if (B == 0 || a.n_slots == 0) return;
	TCNN_CHECK(a.pts_per_chunk == (GRID_BIN_RECS >> D) && a.n_chunks == div_round_up(B, a.pts_per_chunk), "grid bin: chunk plan mismatch");
	const _Float16* dy = (const _Float16*)dLdy16;
	const uint32_t hg = hash_grid ? 1u : 0u, in = (uint32_t)interp;
	switch (D) {
		case 2: grid_bin_f<2>(st, F, h, dy_layout, dy_stride, B, pos, pos_stride, dy, levels, hg, in, a, go); break;
		case 3: grid_bin_f<3>(st, F, h, dy_layout, dy_stride, B, pos, pos_stride, dy, levels, hg, in, a, go); break;
		case 4: grid_bin_f<4>(st, F, h, dy_layout, dy_stride, B, pos, pos_stride, dy, levels, hg, in, a, go); break;
		default: throw std::runtime_error("GridEncoding: number of input dims must be 2, 3 or 4");
	}
	TCNN_HIP_CHECK(hipGetLastError());
}

template <uint32_t NC, uint32_t F>
static void grid_acc_t(hipStream_t st, int layout, uint32_t dys, uint32_t B, const _Float16* dy, const LevelInfo* lv, const GridBinArgs& a,
                       float* grad32, const GridAccAdam* ad) {
	static uint64_t done = 0;
	set_dyn_lds((const void*)k_grid_acc<NC, F>, (int)GRID_ACC_LDS_BYTES, done);
	GridAccAdam adv{};
	if (ad) adv = *ad;
	TCNN_CHECK(a.acc_lds_bytes <= GRID_ACC_LDS_BYTES, "grid acc: slice exceeds the LDS budget");
	TCNN_CHECK(!ad || (ad->param_base % 4 == 0 && ((uintptr_t)ad->buf.w32 & 15) == 0 && ((uintptr_t)ad->buf.w16 & 7) == 0),
	           "grid acc: Adam buffers must be 16-byte aligned with a parameter base that is a multiple of 4");
	hipLaunchKernelGGL((k_grid_acc<NC, F>), dim3(a.n_buckets), dim3(ACC_THREADS), a.acc_lds_bytes, st, layout, B, dy, dys, lv, a, grad32, adv,
	                   ad ? 1 : 0);
}

template <uint32_t NC>
static void grid_acc_f(hipStream_t st, uint32_t F, int layout, uint32_t dys, uint32_t B, const _Float16* dy, const LevelInfo* lv,
                       const GridBinArgs& a, float* grad32, const GridAccAdam* ad) {
	switch (F) {
		case 1: grid_acc_t<NC, 1>(st, layout, dys, B, dy, lv, a, grad32, ad); break;
		case 2: grid_acc_t<NC, 2>(st, layout, dys, B, dy, lv, a, grad32, ad); break;
		case 4: grid_acc_t<NC, 4>(st, layout, dys, B, dy, lv, a, grad32, ad); break;
		case 8: grid_acc_t<NC, 8>(st, layout, dys, B, dy, lv, a, grad32, ad); break;
		default: throw std::runtime_error("GridEncoding: n_features_per_level must be 1, 2, 4 or 8");
	}
}

void launch_grid_acc(hipStream_t st, uint32_t D, uint32_t F, uint32_t B, const void* dLdy16, int dy_layout, uint32_t dy_stride,
                     const LevelInfo* levels, const GridBinArgs& a, float* grad32, const GridAccAdam* adam) {
	if (a.n_slots == 0 || a.n_buckets == 0) return;
	const _Float16* dy = (const _Float16*)dLdy16;
	switch (D) {
		case 2: grid_acc_f<4>(st, F, dy_layout, dy_stride, B, dy, levels, a, grad32, adam); break;
		case 3: grid_acc_f<8>(st, F, dy_layout, dy_stride, B, dy, levels, a, grad32, adam); break;
		case 4: grid_acc_f<16>(st, F, dy_layout, dy_stride, B, dy, levels, a, grad32, adam); break;
		default: throw std::runtime_error("GridEncoding: number of input dims must be 2, 3 or 4");
	}
	TCNN_HIP_CHECK(hipGetLastError());
}

}  // namespace tcnn_amd
