// grid_device.h -- multiresolution grid helpers for gfx950 kernels.
//
// Semantics follow the reference exactly where they decide *which* table entry is touched and how
// the forward interpolation rounds:
//   pos_fract            reference common_device.h:841-868 (pos = fmaf(scale, x, 0.5))
//   grid_index / hashes  reference common_device.h:631-707 (stride loop, hash, % hashmap_size)
//   corner order/weights reference grid.h:144-163 (fp32 weight product, (half)w, fp16 FMA chain)
// The modulo by a runtime table size is specialised: power-of-two sizes (every hashed level) use a
// mask, dense levels only divide in the rare wrap-around case.
#pragma once

#include "common.h"

namespace tcnn_amd {

// Packed fp16 FMA with ONE rounding (CUDA __hfma2 semantics, reference grid.h:162 / vec.h:370-376):
// llvm.fma on <2 x half> is single-rounded by definition, so hipcc must select v_pk_fma_f16 (the
// double-rounding v_fma_mix forms only arise from fp32 arithmetic truncated to fp16, which this
// is not; tests/test_isa_rounding.py rejects any mix form in the library). No inline asm: the
// compiler sees the instruction and pads its MFMA hazards itself (tests/test_isa_hazards.py).
__device__ __forceinline__ h2 pk_fma_f16(h2 a, h2 b, h2 c) { return __builtin_elementwise_fma(a, b, c); }

struct LevelInfo {
	float scale;
	uint32_t res;
	uint32_t offset;  // entries
	uint32_t size;    // entries
};

template <HashType H>
__device__ __forceinline__ uint32_t hash_prime(uint32_t d) {
	if constexpr (H == HashType::Prime) {
		constexpr uint32_t P[7] = {1958374283u, 2654435761u, 805459861u, 3674653429u, 2097192037u, 1434869437u, 2165219737u};
		return P[d];
	} else if constexpr (H == HashType::ReversedPrime) {
		constexpr uint32_t P[7] = {2165219737u, 1434869437u, 2097192037u, 3674653429u, 805459861u, 2654435761u, 1958374283u};
		return P[d];
	} else {
		constexpr uint32_t P[7] = {1u, 2654435761u, 805459861u, 3674653429u, 2097192037u, 1434869437u, 2165219737u};
		return P[d];
	}
}

template <uint32_t D, HashType H>
__device__ __forceinline__ uint32_t grid_index(bool hash_grid, uint32_t size, uint32_t res, const uint32_t* pg) {
	uint32_t stride = 1, index = 0;
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) {
		if (stride > size) break;
		index += pg[d] * stride;
		stride *= res;
	}
	if (hash_grid && size < stride) {
		uint32_t h = 0;
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) h ^= pg[d] * hash_prime<H>(d);
		index = h;
	}
	// index % size (common_device.h:706) without an integer division: hashed levels have
	// power-of-two sizes; a dense level's index is < res^D + res^(D-1) + ... < 2 * size, so one
	// conditional subtraction is exact; only tiled grids (size capped at base^D) may need more.
	if ((size & (size - 1)) == 0) return index & (size - 1);
	if (index >= size) {
		index -= size;
		if (index >= size) index %= size;
	}
	return index;
}

__device__ __forceinline__ void pos_fract(float x, float scale, Interp interp, float& pos, uint32_t& grid) {
	float p = __builtin_fmaf(scale, x, 0.5f);
	float t = floorf(p);
	grid = (uint32_t)(int)t;
	p -= t;
	if (interp == Interp::Smoothstep) p = p * p * __builtin_fmaf(-2.0f, p, 3.0f);
	pos = p;
}

// max_level in levels for point i: (max_level * num_grid_features) / F (grid.h:69-73)
__device__ __forceinline__ float grid_max_level(const GridOpts& o, uint32_t i, uint32_t F) {
	const float ml = o.max_level_gpu ? o.max_level_gpu[i] : o.max_level;
	return (ml * (float)o.n_features) / (float)F;
}

// random_val(1337, idx) (common_device.h:333-337): pcg32{1337} (initseq 1, pcg32.h:45), advance(idx),
// next_float() -- pcg32.h:53-69, 100-110, 139-158.
__device__ __forceinline__ float random_val_1337(uint32_t idx) {
	constexpr uint64_t MULT = 0x5851f42d4c957f2dULL, INC = (1ull << 1) | 1u;
	uint64_t state = 0u;
	state = state * MULT + INC;
	state += 1337u;
	state = state * MULT + INC;
	uint64_t cur_mult = MULT, cur_plus = INC, acc_mult = 1u, acc_plus = 0u;
	for (uint64_t delta = idx; delta > 0; delta >>= 1) {
		if (delta & 1u) {
			acc_mult *= cur_mult;
			acc_plus = acc_plus * cur_mult + cur_plus;
		}
		cur_plus = (cur_mult + 1u) * cur_plus;
		cur_mult *= cur_mult;
	}
	const uint64_t old = acc_mult * state + acc_plus;
	const uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
	const uint32_t rot = (uint32_t)(old >> 59u);
	const uint32_t u = ((xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31))) >> 9 | 0x3f800000u;
	return __builtin_bit_cast(float, u) - 1.0f;
}

// Corner indices (absolute entry index) and fp16 weights of one level; no memory access, so a
// caller can issue the gathers of many levels back to back before consuming any of them.
template <uint32_t D, HashType H>
__device__ __forceinline__ void level_corners(const LevelInfo& li, bool hash_grid, Interp interp, const float* x,
                                              uint32_t* idx, _Float16* w16) {
	float pos[D];
	uint32_t pg[D];
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) pos_fract(x[d], li.scale, interp, pos[d], pg[d]);
	constexpr uint32_t NC = 1u << D;
	if (interp == Interp::Nearest) {
		const uint32_t i0 = li.offset + grid_index<D, H>(hash_grid, li.size, li.res, pg);
#pragma unroll
		for (uint32_t c = 0; c < NC; ++c) { idx[c] = i0; w16[c] = (_Float16)(c == 0 ? 1.0f : 0.0f); }
		return;
	}
#pragma unroll
	for (uint32_t c = 0; c < NC; ++c) {
		float w = 1.0f;
		uint32_t local[D];
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) {
			if ((c & (1u << d)) == 0) { w *= 1.0f - pos[d]; local[d] = pg[d]; }
			else { w *= pos[d]; local[d] = pg[d] + 1; }
		}
		w16[c] = f16_rn(w);
		idx[c] = li.offset + grid_index<D, H>(hash_grid, li.size, li.res, local);
	}
}

// Linear interpolation of one level for F == 2 features (one half2 per table entry). Gathers are
// issued together before the fp16 FMA chain so their latencies overlap.
template <uint32_t D, HashType H>
__device__ __forceinline__ h2 encode_level_f2(const uint32_t* __restrict__ table_u32, const LevelInfo& li,
                                              bool hash_grid, Interp interp, const float* x) {
	float pos[D];
	uint32_t pg[D];
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) pos_fract(x[d], li.scale, interp, pos[d], pg[d]);
	if (interp == Interp::Nearest) {
		uint32_t idx = grid_index<D, H>(hash_grid, li.size, li.res, pg);
		uint32_t v = table_u32[li.offset + idx];
		return __builtin_bit_cast(h2, v);
	}
	constexpr uint32_t NC = 1u << D;
	uint32_t v[NC];
	_Float16 w16[NC];
	float wf[NC];
#pragma unroll
	for (uint32_t c = 0; c < NC; ++c) {
		float w = 1.0f;
		uint32_t local[D];
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) {
			if ((c & (1u << d)) == 0) { w *= 1.0f - pos[d]; local[d] = pg[d]; }
			else { w *= pos[d]; local[d] = pg[d] + 1; }
		}
		// converted in pairs below (f16_rn_pairs: v_cvt_pk_f16_f32, no fused mix rounding; pinned for
		// every kernel by tests/test_isa_rounding.py); an f16_rn barrier per weight costs the fused
		// kernel ~10% by serialising the weight / gather schedule
		wf[c] = w;
		v[c] = table_u32[li.offset + grid_index<D, H>(hash_grid, li.size, li.res, local)];
	}
	f16_rn_pairs(wf, w16);
	h2 r = {(_Float16)0.0f, (_Float16)0.0f};
#pragma unroll
	for (uint32_t c = 0; c < NC; ++c) {
		h2 wv = {w16[c], w16[c]};
		r = pk_fma_f16(wv, __builtin_bit_cast(h2, v[c]), r);
	}
	return r;
}

// grid_index for positions inside [0, 1] on a level that is hashed with a power-of-two size or dense
// (res^D <= size): there the dense index is below 2 * size, so `% size` is one conditional
// subtraction and the whole computation is branch-free -- the compiler can then issue the gathers of
// several levels before consuming any of them. Same result as grid_index under those conditions
// (the caller checks them: GridEncodingHost::inrange_index_ok and a wave-wide position test).
template <uint32_t D, HashType H>
__device__ __forceinline__ uint32_t grid_index_inrange(bool hash_grid, uint32_t size, uint32_t res, const uint32_t* pg) {
	uint32_t stride = 1, dense = 0;
	bool brk = false;
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) {  // the reference's stride loop, its break as a predicate
		brk = brk || stride > size;
		dense = brk ? dense : dense + pg[d] * stride;
		stride = brk ? stride : stride * res;
	}
	uint32_t h = 0;
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) h ^= pg[d] * hash_prime<H>(d);
	const bool hashed = hash_grid && size < stride;
	const uint32_t dm = dense >= size ? dense - size : dense;
	return hashed ? (h & (size - 1)) : dm;
}

// What encode_level_f2_inrange needs of a level, independent of the point: computed once per level
// and shared by every point a lane encodes at that level (the fused kernel's two sample tiles).
template <uint32_t D>
struct LevelConsts {
	float scale;
	uint32_t size, hmask, obytes, m;  // m: all ones where the level is hashed (see below)
	uint32_t sd[D];                   // dense stride of each dimension (res^d)
};

// grid_index_inrange with everything that does not depend on the corner hoisted: per dimension the
// hash term pg*P and the dense term pg*res^d for both corner offsets ((pg + 1) * k = pg * k + k, also
// modulo 2^32). Under GridEncodingHost::inrange_index_ok a level whose index is used densely has
// res^D <= size (the stride loop never breaks), and its corner indices stay below 2 * size. The
// hashed / dense choice is per lane (lanes hold different levels), so it is a bit select on an
// opaque mask: written as a C select, the compiler sank the two index computations into divergent
// branches (exec-mask regions around every corner), which also kept it from issuing one level's
// gathers before the previous level's FMA chain.
template <uint32_t D>
__device__ __forceinline__ LevelConsts<D> level_consts(const LevelInfo& li, bool hash_grid) {
	LevelConsts<D> c;
	uint32_t stride = 1;
	bool brk = false;
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) {
		c.sd[d] = stride;
		brk = brk || stride > li.size;  // the reference's stride loop (common_device.h:691-697)
		stride = brk ? stride : stride * li.res;
	}
	uint32_t m = (hash_grid && li.size < stride) ? 0xffffffffu : 0u;
	asm("" : "+v"(m));
	c.m = m;
	c.scale = li.scale;
	c.size = li.size;
	c.hmask = li.size - 1;
	c.obytes = li.offset << 2;
	return c;
}

template <uint32_t D, HashType H>
__device__ __forceinline__ h2 encode_level_f2_inrange(const uint32_t* __restrict__ table_u32, const LevelConsts<D>& lc, const float* x) {
	float pos[D];
	uint32_t pg[D];
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) pos_fract(x[d], lc.scale, Interp::Linear, pos[d], pg[d]);
	constexpr uint32_t NC = 1u << D;
	uint32_t th[D][2], td[D][2];
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) {
		th[d][0] = pg[d] * hash_prime<H>(d);
		th[d][1] = th[d][0] + hash_prime<H>(d);
		td[d][0] = pg[d] * lc.sd[d];
		td[d][1] = td[d][0] + lc.sd[d];
	}
	const uint32_t m = lc.m, hmask = lc.hmask, obytes = lc.obytes;
	uint32_t v[NC];
	_Float16 w16[NC];
	float wf[NC];
#pragma unroll
	for (uint32_t c = 0; c < NC; ++c) {
		float w = 1.0f;
		uint32_t h = 0, dn = 0;
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) {
			const uint32_t b = (c >> d) & 1u;
			w *= b ? pos[d] : 1.0f - pos[d];
			h ^= th[d][b];
			dn += td[d][b];
		}
		const uint32_t dm = __builtin_elementwise_min(dn, dn - lc.size);  // dn % size for dn < 2 size
		uint32_t idx = ((h & hmask) & m) | (dm & ~m);
#ifdef TCNN_DIAG_GATHER_MASK  // diagnostic builds only (wrong results): gathers confined to a few cache lines
		idx &= TCNN_DIAG_GATHER_MASK;
#endif
		wf[c] = w;  // as encode_level_f2
		v[c] = *(const uint32_t*)((const char*)table_u32 + (obytes + (idx << 2)));
	}
	f16_rn_pairs(wf, w16);
	h2 r = {(_Float16)0.0f, (_Float16)0.0f};
#pragma unroll
	for (uint32_t c = 0; c < NC; ++c) {
		h2 wv = {w16[c], w16[c]};
		r = pk_fma_f16(wv, __builtin_bit_cast(h2, v[c]), r);
	}
	return r;
}

// Lane-pair gathers (r04). The vector L1 costs one tag lookup per distinct cache line of an
// instruction (tools/gather_bench.hip, profiles/r04_gather_bench.json: 64 random lines per
// instruction take twice as long as 32 lines shared by lane pairs, whichever lanes share). A
// point's two x-neighbour corners sit in one line (CoherentPrime's x term is x * 1; dense levels
// are x-contiguous), so lanes L and L^1 fetch them in the same instruction: per level, the pair
// gathers point A (the even lane's sample) then point B (the odd lane's), each lane the corners of
// its own x parity `par`, then swaps half of the values (DPP quad_perm [1,0,3,2]) so each lane holds
// all 2^D corners of its own point and runs the same fp16 FMA chain in the same corner order as
// encode_level_f2_inrange -- bit-identical, with half the L1 line work.
// xA / xB: the positions of the even / odd lane's sample (the lane's own is xB if par, else xA).
// The whole wave must be active (the callers' in-range branch is wave-uniform).
// Coarse dense levels staged in LDS (r04): levels 0..k-1 of the table prefix, while they are dense
// (not hashed) and their entries fit `budget_bytes`; the fused kernels then read those levels
// through a per-lane table pointer into LDS (a flat load: lanes of one instruction may mix LDS and
// global levels). Every sample touches every level, so the small dense tables -- evicted from the
// 32 KB L1 by the hashed levels' stream -- otherwise cost two L2 requests per sample and level.
// Returns the staged entry count (0: none); `k` = the number of staged levels.
template <uint32_t D>
__device__ __forceinline__ uint32_t stage_dense_levels(uint32_t* __restrict__ sT, const uint32_t* __restrict__ table, const LevelInfo* sLvl,
                                                       uint32_t n_levels, bool hash_grid, uint32_t budget_bytes, int tid, int nthreads,
                                                       uint32_t& k) {
	uint32_t entries = 0;
	k = 0;
	for (uint32_t l = 0; l < n_levels; ++l) {
		const LevelInfo li = sLvl[l];
		uint64_t full = 1;
		for (uint32_t d = 0; d < D; ++d) full *= li.res;
		const bool dense = !hash_grid || full <= li.size;
		if (!dense || li.offset != entries || (uint64_t)(li.offset + li.size) * 4 > budget_bytes) break;
		entries = li.offset + li.size;
		k = l + 1;
	}
	if (((uintptr_t)table & 15) == 0) {
		for (uint32_t j = tid; j < entries / 4; j += nthreads) ((uint4*)sT)[j] = ((const uint4*)table)[j];
		for (uint32_t j = entries / 4 * 4 + tid; j < entries; j += nthreads) sT[j] = table[j];
	} else {
		for (uint32_t j = tid; j < entries; j += nthreads) sT[j] = table[j];
	}
	return entries;
}

__device__ __forceinline__ uint32_t dpp_swap_pair(uint32_t v) {
	return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ float dpp_swap_pair(float v) { return __builtin_bit_cast(float, dpp_swap_pair(__builtin_bit_cast(uint32_t, v))); }

template <uint32_t D, HashType H>
__device__ __forceinline__ h2 encode_level_f2_pair(const uint32_t* __restrict__ table_u32, const LevelConsts<D>& lc, const float* xA,
                                                   const float* xB, uint32_t par) {
	constexpr uint32_t NC = 1u << D, NR = NC / 2;
	const uint32_t m = lc.m, hmask = lc.hmask, obytes = lc.obytes;
	float posA[D], posB[D];
	uint32_t vA[NR], vB[NR];
	// the corners with x bit = par of one point: rows r = corner >> 1
	auto gather_rows = [&](const float* x, float (&pos)[D], uint32_t (&v)[NR]) {
		uint32_t pg[D];
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) pos_fract(x[d], lc.scale, Interp::Linear, pos[d], pg[d]);
		uint32_t th[D][2], td[D][2];
		th[0][0] = th[0][1] = (pg[0] + par) * hash_prime<H>(0);
		td[0][0] = td[0][1] = (pg[0] + par) * lc.sd[0];
#pragma unroll
		for (uint32_t d = 1; d < D; ++d) {
			th[d][0] = pg[d] * hash_prime<H>(d);
			th[d][1] = th[d][0] + hash_prime<H>(d);
			td[d][0] = pg[d] * lc.sd[d];
			td[d][1] = td[d][0] + lc.sd[d];
		}
#pragma unroll
		for (uint32_t r = 0; r < NR; ++r) {
			uint32_t h = th[0][0], dn = td[0][0];
#pragma unroll
			for (uint32_t d = 1; d < D; ++d) {
				const uint32_t b = (r >> (d - 1)) & 1u;
				h ^= th[d][b];
				dn += td[d][b];
			}
			const uint32_t dm = __builtin_elementwise_min(dn, dn - lc.size);  // dn % size for dn < 2 size
			const uint32_t idx = ((h & hmask) & m) | (dm & ~m);
			v[r] = *(const uint32_t*)((const char*)table_u32 + (obytes + (idx << 2)));
		}
	};
	gather_rows(xA, posA, vA);
	gather_rows(xB, posB, vB);
	uint32_t v[NC];
#pragma unroll
	for (uint32_t r = 0; r < NR; ++r) {
		const uint32_t recv = dpp_swap_pair(par ? vA[r] : vB[r]);  // the partner's corners of my point
		v[2 * r] = par ? recv : vA[r];
		v[2 * r + 1] = par ? vB[r] : recv;
	}
	_Float16 w16[NC];
	float wf[NC];
#pragma unroll
	for (uint32_t c = 0; c < NC; ++c) {
		float w = 1.0f;
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) {
			const float p = par ? posB[d] : posA[d];
			w *= ((c >> d) & 1u) ? p : 1.0f - p;
		}
		wf[c] = w;  // as encode_level_f2
	}
	f16_rn_pairs(wf, w16);
	h2 res = {(_Float16)0.0f, (_Float16)0.0f};
#pragma unroll
	for (uint32_t c = 0; c < NC; ++c) {
		h2 wv = {w16[c], w16[c]};
		res = pk_fma_f16(wv, __builtin_bit_cast(h2, v[c]), res);
	}
	return res;
}

// encode_level_f2_pair in two halves (r06, the fused kernel's small-batch schedule): _gather issues the
// lane's 2 NR corner loads and returns them unconsumed, so a caller can have every level's loads in
// flight before the first combine; _combine is the rest of encode_level_f2_pair -- the same DPP swap,
// weights and fp16 FMA chain, bit-identical.
template <uint32_t NR>
struct PairGather {
	uint32_t vA[NR], vB[NR];
};
template <uint32_t D, HashType H>
__device__ __forceinline__ PairGather<(1u << D) / 2> encode_level_f2_pair_gather(const uint32_t* __restrict__ table_u32, const LevelConsts<D>& lc,
                                                                                 const float* xA, const float* xB, uint32_t par) {
	constexpr uint32_t NR = (1u << D) / 2;
	const uint32_t m = lc.m, hmask = lc.hmask, obytes = lc.obytes;
	PairGather<NR> g;
#pragma unroll
	for (uint32_t P = 0; P < 2; ++P) {
		const float* x = P ? xB : xA;
		uint32_t pg[D];
		float pos;
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) pos_fract(x[d], lc.scale, Interp::Linear, pos, pg[d]);
		uint32_t th[D][2], td[D][2];
		th[0][0] = th[0][1] = (pg[0] + par) * hash_prime<H>(0);
		td[0][0] = td[0][1] = (pg[0] + par) * lc.sd[0];
#pragma unroll
		for (uint32_t d = 1; d < D; ++d) {
			th[d][0] = pg[d] * hash_prime<H>(d);
			th[d][1] = th[d][0] + hash_prime<H>(d);
			td[d][0] = pg[d] * lc.sd[d];
			td[d][1] = td[d][0] + lc.sd[d];
		}
#pragma unroll
		for (uint32_t r = 0; r < NR; ++r) {
			uint32_t h = th[0][0], dn = td[0][0];
#pragma unroll
			for (uint32_t d = 1; d < D; ++d) {
				const uint32_t b = (r >> (d - 1)) & 1u;
				h ^= th[d][b];
				dn += td[d][b];
			}
			const uint32_t dm = __builtin_elementwise_min(dn, dn - lc.size);
			const uint32_t idx = ((h & hmask) & m) | (dm & ~m);
			(P ? g.vB : g.vA)[r] = *(const uint32_t*)((const char*)table_u32 + (obytes + (idx << 2)));
		}
	}
	return g;
}
template <uint32_t D>
__device__ __forceinline__ h2 encode_level_f2_pair_combine(const PairGather<(1u << D) / 2>& g, float scale, const float* xA, const float* xB,
                                                           uint32_t par) {
	constexpr uint32_t NC = 1u << D, NR = NC / 2;
	float pos[D];
	uint32_t pg;
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) pos_fract(par ? xB[d] : xA[d], scale, Interp::Linear, pos[d], pg);
	uint32_t v[NC];
#pragma unroll
	for (uint32_t r = 0; r < NR; ++r) {
		const uint32_t recv = dpp_swap_pair(par ? g.vA[r] : g.vB[r]);  // the partner's corners of my point
		v[2 * r] = par ? recv : g.vA[r];
		v[2 * r + 1] = par ? g.vB[r] : recv;
	}
	_Float16 w16[NC];
	float wf[NC];
#pragma unroll
	for (uint32_t c = 0; c < NC; ++c) {
		float w = 1.0f;
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) w *= ((c >> d) & 1u) ? pos[d] : 1.0f - pos[d];
		wf[c] = w;
	}
	f16_rn_pairs(wf, w16);
	h2 res = {(_Float16)0.0f, (_Float16)0.0f};
#pragma unroll
	for (uint32_t c = 0; c < NC; ++c) {
		h2 wv = {w16[c], w16[c]};
		res = pk_fma_f16(wv, __builtin_bit_cast(h2, v[c]), res);
	}
	return res;
}

template <uint32_t D, HashType H>
__device__ __forceinline__ h2 encode_level_f2_inrange(const uint32_t* __restrict__ table_u32, const LevelInfo& li, bool hash_grid,
                                                      const float* x) {
	return encode_level_f2_inrange<D, H>(table_u32, level_consts<D>(li, hash_grid), x);
}

// F fp16 features of one table entry / one point-level
template <uint32_t F>
struct HVec { _Float16 v[F]; };

// dL/dy of point i, level `level` (F features) in one of the grid backward's layouts:
// 0 = level-major feature pairs [l][i][F], 1 = SoA [(l*F+f)*B + i] (reference RM), 2 = AoS
// [i*stride + l*F + f] (reference CM)
template <uint32_t F>
__device__ __forceinline__ void load_dy(int layout, const _Float16* __restrict__ dLdy, uint32_t dy_stride, uint32_t level, uint32_t B,
                                        uint32_t i, float* dy) {
	if (layout == 0) {  // level-major feature pairs [l][i][F]
		const HVec<F> v = ((const HVec<F>*)dLdy)[(size_t)level * B + i];
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) dy[f] = (float)v.v[f];
	} else if (layout == 1) {  // SoA [(l*F+f)*B + i] (reference RM layout)
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) dy[f] = (float)dLdy[(size_t)(level * F + f) * B + i];
	} else {  // AoS [i*stride + l*F + f] (reference CM layout)
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) dy[f] = (float)dLdy[(size_t)i * dy_stride + level * F + f];
	}
}

// The raw fp16 bits of dL/dy of point i, level `level` (F <= 2 features, feature f in bits
// [16f, 16f + 16)), same layouts as load_dy.
template <uint32_t F>
__device__ __forceinline__ uint32_t load_dy_bits(int layout, const _Float16* __restrict__ dLdy, uint32_t dy_stride, uint32_t level,
                                                 uint32_t B, uint32_t i) {
	static_assert(F <= 2, "load_dy_bits: F <= 2");
	const uint16_t* d16 = (const uint16_t*)dLdy;
	if (layout == 0) {
		if constexpr (F == 2) return ((const uint32_t*)dLdy)[(size_t)level * B + i];
		else return d16[(size_t)level * B + i];
	}
	uint32_t r = 0;
#pragma unroll
	for (uint32_t f = 0; f < F; ++f)
		r |= (uint32_t)(layout == 1 ? d16[(size_t)(level * F + f) * B + i] : d16[(size_t)i * dy_stride + level * F + f]) << (16 * f);
	return r;
}

__device__ __forceinline__ float dy_bits_feature(uint32_t bits, uint32_t f) {
	return (float)__builtin_bit_cast(_Float16, (uint16_t)(bits >> (16 * f)));
}

}  // namespace tcnn_amd
