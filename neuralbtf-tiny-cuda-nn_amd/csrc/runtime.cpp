// runtime.cpp -- host runtime: JSON config surface, parameter init, trainer orchestration.
#include "runtime.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstring>
#include <limits>
#include <random>

namespace tcnn_amd {

// ------------------------------------------------------------------------------------------
// PCG32 (stream semantics of dependencies/pcg32/pcg32.h)
// ------------------------------------------------------------------------------------------
static constexpr uint64_t PCG32_MULT = 0x5851f42d4c957f2dULL;

void Pcg32::seed(uint64_t initstate, uint64_t initseq) {
	state = 0u;
	inc = (initseq << 1u) | 1u;
	next_uint();
	state += initstate;
	next_uint();
}

uint32_t Pcg32::next_uint() {
	uint64_t old = state;
	state = old * PCG32_MULT + inc;
	uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
	uint32_t rot = (uint32_t)(old >> 59u);
	return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
}

float Pcg32::next_float() {
	uint32_t u = (next_uint() >> 9) | 0x3f800000u;
	float f;
	std::memcpy(&f, &u, 4);
	return f - 1.0f;
}

void Pcg32::advance(int64_t delta_) {
	uint64_t cur_mult = PCG32_MULT, cur_plus = inc, acc_mult = 1u, acc_plus = 0u;
	uint64_t delta = (uint64_t)delta_;
	while (delta > 0) {
		if (delta & 1) {
			acc_mult *= cur_mult;
			acc_plus = acc_plus * cur_mult + cur_plus;
		}
		cur_plus = (cur_mult + 1) * cur_plus;
		cur_mult *= cur_mult;
		delta /= 2;
	}
	state = acc_mult * state + acc_plus;
}

// generate_random_uniform's strided order (reference random.h:39-70), evaluated on the host.
static void strided_uniform(Pcg32& rng, size_t n, float* out, float lo, float hi) {
	const size_t n_gen = 4;
	const size_t n_thr = (n + n_gen - 1) / n_gen;
	const size_t n_threads = (n_thr + 127) / 128 * 128;
	const float range = hi - lo;
	for (size_t i = 0; i < n_threads; ++i) {  // all launched threads write, also those past n_thr (random.h:41-54)
		Pcg32 r = rng;
		r.advance((int64_t)(i * n_gen));
		for (size_t j = 0; j < n_gen; ++j) {
			size_t idx = i + n_threads * j;
			if (idx >= n) break;
			out[idx] = std::fma(r.next_float(), range, lo);
		}
	}
	rng.advance((int64_t)n);
}

// ------------------------------------------------------------------------------------------
// DevBuf
// ------------------------------------------------------------------------------------------
DevBuf::~DevBuf() { release(); }

void DevBuf::release() {
	if (p) (void)hipFree(p);
	p = nullptr;
	bytes = 0;
}

void DevBuf::reserve(size_t n) {
	if (n <= bytes && p) return;
	release();
	if (n == 0) n = 16;
	TCNN_HIP_CHECK(hipMalloc(&p, n));
	bytes = n;
	static const bool poison = std::getenv("TCNN_DEBUG_POISON") != nullptr;  // NaN-fill new buffers (finds reads of unwritten memory)
	if (poison) TCNN_HIP_CHECK(hipMemset(p, 0xff, n));
}

EngineSwitches EngineSwitches::from_env() {
	EngineSwitches s;
	auto on = [](const char* n) { return std::getenv(n) != nullptr; };
	s.no_fused_grid = on("TCNN_NO_FUSED_GRID");
	s.no_tile_engine = on("TCNN_NO_TILE_ENGINE");
	s.no_inrange_index = on("TCNN_NO_INRANGE_INDEX");
	s.split_encode = on("TCNN_SPLIT_ENCODE");
	s.no_forward_keep = on("TCNN_NO_FORWARD_KEEP");
	s.split_forward = on("TCNN_SPLIT_FORWARD");
	const char* bin = std::getenv("TCNN_GRID_BIN");
	s.grid_bin_all = bin && std::string(bin) == "all";
	if (const char* e = std::getenv("TCNN_GRID_BWD_CHUNKS"))
		if (std::atoi(e) > 0) s.grid_bwd_chunks = (uint32_t)std::atoi(e);
	if (const char* e = std::getenv("TCNN_GRID_BWD_RANGES"))
		if (std::atoi(e) > 0) s.grid_bwd_ranges = (uint32_t)std::atoi(e);
	if (const char* e = std::getenv("TCNN_GRID_BWD_PLAN")) s.grid_bwd_plan = std::string(e) == "feature" ? 1 : (std::string(e) == "range" ? 0 : -1);
	return s;
}

bool ieq(const std::string& a, const std::string& b) {
	if (a.size() != b.size()) return false;
	for (size_t i = 0; i < a.size(); ++i)
		if (std::tolower((unsigned char)a[i]) != std::tolower((unsigned char)b[i])) return false;
	return true;
}

template <typename T>
static T jval(const json& j, const char* key, T dflt) {
	auto it = j.find(key);
	if (it == j.end() || it->is_null()) return dflt;
	return it->get<T>();
}

static bool jhas(const json& j, const char* key) { return j.is_object() && j.find(key) != j.end(); }

// ------------------------------------------------------------------------------------------
// Grid encoding (reference grid.h:652-1208)
// ------------------------------------------------------------------------------------------
static uint32_t powi_u32(uint32_t base, uint32_t exp) {
	uint32_t r = 1;
	for (uint32_t i = 0; i < exp; ++i) r *= base;
	return r;
}

GridEncodingHost::GridEncodingHost(uint32_t n_dims, const json& enc) {
	const std::string otype = jval<std::string>(enc, "otype", "Grid");
	const std::string default_type = ieq(otype, "TiledGrid") ? "Tiled" : (ieq(otype, "DenseGrid") ? "Dense" : "Hash");
	const uint32_t F = jval<uint32_t>(enc, "n_features_per_level", 2u);
	TCNN_CHECK(F == 1 || F == 2 || F == 4 || F == 8, "GridEncoding: n_features_per_level must be 1, 2, 4, or 8.");
	uint32_t n_feat;
	if (jhas(enc, "n_features") || jhas(enc, "n_grid_features")) {
		n_feat = jhas(enc, "n_features") ? enc["n_features"].get<uint32_t>() : enc["n_grid_features"].get<uint32_t>();
		TCNN_CHECK(!jhas(enc, "n_levels"), "GridEncoding: may not specify n_features and n_levels simultaneously (one determines the other)");
	} else {
		n_feat = F * jval<uint32_t>(enc, "n_levels", 16u);
	}
	TCNN_CHECK(n_feat % F == 0, "GridEncoding: n_features must be a multiple of n_features_per_level");
	const uint32_t L = n_feat / F;
	TCNN_CHECK(L >= 1 && L <= MAX_LEVELS, "GridEncoding: too many levels");
	const std::string type = jval<std::string>(enc, "type", default_type);
	GridType gt;
	if (ieq(type, "Hash")) gt = GridType::Hash;
	else if (ieq(type, "Dense")) gt = GridType::Dense;
	else if (ieq(type, "Tiled")) gt = GridType::Tiled;
	else throw std::runtime_error("GridEncoding: invalid grid type " + type);
	const uint32_t base = jval<uint32_t>(enc, "base_resolution", 16u);
	const float default_scale = gt == GridType::Dense ? std::exp(std::log(256.0f / (float)base) / (float)(L - 1)) : 2.0f;
	const std::string interp = jval<std::string>(enc, "interpolation", "Linear");
	const std::string hash = jval<std::string>(enc, "hash", "CoherentPrime");
	TCNN_CHECK(n_dims >= 2 && n_dims <= 4, "GridEncoding: number of input dims must be 2, 3 or 4.");

	desc.n_pos_dims = n_dims;
	desc.n_features_per_level = F;
	desc.n_levels = L;
	desc.log2_hashmap_size = jval<uint32_t>(enc, "log2_hashmap_size", 19u);
	desc.base_resolution = base;
	desc.per_level_scale = jval<float>(enc, "per_level_scale", default_scale);
	desc.grid_type = gt;
	if (ieq(hash, "Prime")) desc.hash_type = HashType::Prime;
	else if (ieq(hash, "CoherentPrime")) desc.hash_type = HashType::CoherentPrime;
	else if (ieq(hash, "ReversedPrime")) desc.hash_type = HashType::ReversedPrime;
	else throw std::runtime_error("GridEncoding: unsupported hash type " + hash);
	if (ieq(interp, "Nearest")) desc.interp = Interp::Nearest;
	else if (ieq(interp, "Linear")) desc.interp = Interp::Linear;
	else if (ieq(interp, "Smoothstep")) desc.interp = Interp::Smoothstep;
	else throw std::runtime_error("GridEncoding: invalid interpolation " + interp);
	stochastic = jval<bool>(enc, "stochastic_interpolation", false);
	n_features = n_feat;

	// offset table, grid.h:688-719 (host log2/exp2 in float, as the reference's host code)
	const float log2_scale = std::log2(desc.per_level_scale);
	uint32_t offset = 0;
	levels.resize(L);
	for (uint32_t l = 0; l < L; ++l) {
		const float scale = exp2f((float)l * log2_scale) * (float)base - 1.0f;
		const uint32_t res = (uint32_t)ceilf(scale) + 1;
		const uint32_t max_params = std::numeric_limits<uint32_t>::max() / 2;
		uint32_t params = std::pow((float)res, (float)n_dims) > (float)max_params ? max_params : powi_u32(res, n_dims);
		params = (params + 7u) / 8u * 8u;
		if (gt == GridType::Tiled) params = std::min(params, powi_u32(base, n_dims));
		else if (gt == GridType::Hash) params = std::min(params, 1u << desc.log2_hashmap_size);
		levels[l] = LevelInfo{scale, res, offset, params};
		log_debug("GridEncoding at level " + std::to_string(l) + ": resolution=" + std::to_string(res) +
		          " params_in_level=" + std::to_string(params));  // grid.h:717
		offset += params;
	}
	n_params = offset * F;

	// Backward plan. A level whose F features fit the LDS budget is one LDS item; else, when one
	// feature fits, one item per feature group (config_hash's 2^15-entry hashed levels: two items);
	// levels with even one feature over the budget -- and every level after them, so the binned
	// levels are a suffix of the parameter vector -- go through the binned backward (grid_bin.hip).
	// TCNN_GRID_BIN=all bins every level that does not fit whole (tuning switch).
	const uint32_t S = grid_bwd_slot_budget();
	const bool bin_all = sw.grid_bin_all;
	first_binned = L;
	for (uint32_t l = 0; l < L; ++l) {
		const uint64_t need = bin_all ? (uint64_t)levels[l].size * F : (uint64_t)levels[l].size;
		if (need > S) { first_binned = l; break; }
	}
	n_lds_params = (first_binned < L ? levels[first_binned].offset : offset) * F;
	// Two work plans for the LDS levels (r06), chosen per launch (plan_for). Both: a level whose F
	// features fit the budget is one item; the others split --
	//   PLAN_RANGE:   a hashed power-of-two level into entry ranges holding all F features: the chunk
	//                 slabs are in parameter order (Adam and the slab sums read them without the map),
	//                 the packed-pair LDS adds of MODE 0 apply for F = 2;
	//   PLAN_FEATURE: into feature groups (r05): each writes a feature-group-major run, read back
	//                 through GridSlabMap.
	// Measured (profiles/r06_grid_plan_ab.json): the range plan takes 2^15 / 2^18-point steps 2 us /
	// 1.4 % faster (Adam 15.0 -> 13.0 us at 2^18), the feature plan is 25 % faster in configs[3]'s
	// 2^20-point backward, whose chunks run in several rounds.
	GridSlabMap map{};
	map.n_levels = std::max(1u, first_binned);
	while ((1u << map.log2F) < F) ++map.log2F;
	for (int plan = 0; plan < 2; ++plan) {
		std::vector<GridSlice>& out = plans[plan].slices;
		std::vector<GridSlice> single;
		for (uint32_t l = 0; l < first_binned; ++l) {
			const uint32_t size = levels[l].size;
			map.pbase[l] = levels[l].offset * F;
			map.size[l] = size;
			if (plan == PLAN_FEATURE) map.nf[l] = F;
			if ((uint64_t)size * F <= S) {
				out.push_back(GridSlice{l, 0, size, 0, F});
				continue;
			}
			uint32_t full = 1;
			for (uint32_t d = 0; d < desc.n_pos_dims && full <= size; ++d) full *= levels[l].res;
			const bool hashed_pow2 = gt == GridType::Hash && (size & (size - 1)) == 0 && full > size;
			if (plan == PLAN_RANGE && hashed_pow2) {
				uint32_t R = 1;
				while ((uint64_t)size * F / R > S) R *= 2;
				R = std::max(R, std::min(sw.grid_bwd_ranges, size / 256));  // tuning override (TCNN_GRID_BWD_RANGES)
				const uint32_t len = size / R;
				for (uint32_t r = 0; r < R; ++r) single.push_back(GridSlice{l, r * len, (r + 1) * len, 0, F});
				continue;
			}
			uint32_t nf = F;
			while (nf > 1 && ((uint64_t)size * nf > S || F % nf)) --nf;
			if (plan == PLAN_FEATURE) map.nf[l] = nf;
			else plans[plan].identity = false;  // a non-hashed level split by features: the range plan needs the map too
			for (uint32_t f = 0; f < F; f += nf) single.push_back(GridSlice{l, 0, size, f, nf});
		}
		out.insert(out.end(), single.begin(), single.end());
	}
	plans[PLAN_FEATURE].identity = true;
	for (uint32_t l = 0; l < first_binned; ++l) plans[PLAN_FEATURE].identity = plans[PLAN_FEATURE].identity && map.nf[l] == F;
	if (!plans[PLAN_RANGE].identity) plans[PLAN_RANGE] = plans[PLAN_FEATURE];  // (no hashed split: one plan)
	map.pbase[first_binned] = n_lds_params;
	d_slab_map.reserve(sizeof(GridSlabMap));
	TCNN_HIP_CHECK(hipMemcpy(d_slab_map.p, &map, sizeof(GridSlabMap), hipMemcpyHostToDevice));

	// binned levels: slices of 2^s entries, ~128 per level (one workgroup each in the accumulate
	// pass), within the accumulator budget and GRID_BIN_MAX_SLICES
	const uint32_t max_entries = GRID_ACC_LDS_BYTES / 4 / F;
	for (uint32_t l = first_binned; l < L; ++l) {
		const uint32_t size = levels[l].size;
		uint32_t lg = 0;
		while ((1ull << lg) < size) ++lg;
		uint32_t s = lg > 7 ? lg - 7 : 0;
		s = std::max(s, 9u);
		while ((1u << s) > max_entries) --s;
		TCNN_CHECK(div_round_up(size, 1u << s) <= GRID_BIN_MAX_SLICES,
		           "GridEncoding: level of " + std::to_string(size) + " entries exceeds the binned backward's capacity");
		GridBinLevel b{l, s, div_round_up(size, 1u << s), n_buckets};
		n_buckets += b.n_slices;
		acc_lds_bytes = std::max(acc_lds_bytes, (1u << s) * F * 4);
		bin_levels.push_back(b);
	}
	if (!bin_levels.empty()) {
		d_bin_levels.reserve(bin_levels.size() * sizeof(GridBinLevel));
		TCNN_HIP_CHECK(hipMemcpy(d_bin_levels.p, bin_levels.data(), bin_levels.size() * sizeof(GridBinLevel), hipMemcpyHostToDevice));
	}

	// grid_index_inrange (grid_device.h: the reference stride loop, then a mask or ONE conditional
	// subtraction) is exact for positions in [0, 1] on every level iff hashed levels have
	// power-of-two sizes and the others hold res^D entries (their index is then < 2 size)
	inrange_index_ok = true;
	for (const LevelInfo& li : levels) {
		uint32_t stride = 1;
		for (uint32_t d = 0; d < desc.n_pos_dims; ++d)
			if (stride <= li.size) stride *= li.res;
		uint64_t full = 1;
		for (uint32_t d = 0; d < desc.n_pos_dims; ++d) full = std::min<uint64_t>(full * li.res, 1ull << 40);
		const bool hashed = hash_grid() && li.size < stride;
		if (hashed ? (li.size & (li.size - 1)) != 0 : full > li.size) inrange_index_ok = false;
		if (li.res < 2) inrange_index_ok = false;
	}
	d_levels.reserve(levels.size() * sizeof(LevelInfo));
	TCNN_HIP_CHECK(hipMemcpy(d_levels.p, levels.data(), levels.size() * sizeof(LevelInfo), hipMemcpyHostToDevice));
	for (GridPlan& pl : plans) {
		pl.d_slices.reserve(pl.slices.size() * sizeof(GridSlice));
		TCNN_HIP_CHECK(hipMemcpy(pl.d_slices.p, pl.slices.data(), pl.slices.size() * sizeof(GridSlice), hipMemcpyHostToDevice));
	}
}

void GridEncodingHost::initialize_params(Pcg32& rng, float* out, float scale) const {
	strided_uniform(rng, n_params, out, -1e-4f * scale, 1e-4f * scale);
}

GridBinArgs GridEncodingHost::bin_args(GridBwdBufs& w, uint32_t B) const {
	GridBinArgs a{};
	a.lv = d_bin_levels.as<GridBinLevel>();
	a.n_slots = (uint32_t)bin_levels.size();
	a.n_buckets = n_buckets;
	a.pts_per_chunk = GRID_BIN_RECS >> desc.n_pos_dims;
	a.n_chunks = div_round_up(std::max(B, 1u), a.pts_per_chunk);
	a.acc_lds_bytes = acc_lds_bytes;
	if (a.n_slots) {
		w.recs.reserve((size_t)a.n_slots * a.n_chunks * GRID_BIN_RECS * sizeof(uint2));
		w.dir.reserve((size_t)a.n_buckets * a.n_chunks * sizeof(uint2));
		w.dysum.reserve((size_t)a.n_slots * a.n_chunks * desc.n_features_per_level * sizeof(float));
	}
	a.recs = w.recs.as<uint2>();
	a.dir = w.dir.as<uint2>();
	a.dysum = w.dysum.as<float>();
	return a;
}

void GridEncodingHost::backward_items(hipStream_t st, GridBwdBufs& w, uint32_t B, const float* pos, uint32_t pstride, const void* dy,
                                      int layout, uint32_t dy_stride, const GridBwdEpilogue* ep, uint32_t reserved) const {
	const uint32_t n_chunks = bwd_chunks(B, reserved);
	w.n_chunks = n_chunks;
	w.plan = plan_for(B, reserved);
	const GridPlan& pl = plans[w.plan];
	if (!pl.slices.empty()) w.partial.reserve((size_t)n_chunks * n_lds_params * 4);
	launch_grid_bwd(st, desc.n_pos_dims, desc.n_features_per_level, desc.hash_type, B, pos, pstride, dy, layout, dy_stride,
	                pl.d_slices.as<GridSlice>(), (uint32_t)pl.slices.size(), n_chunks, w.partial.as<float>(), n_lds_params, dev_levels(),
	                hash_grid(), desc.interp, ep, opts(), pl.slices.data(), levels.data(), (uint32_t)levels.size());
}

void GridEncodingHost::backward_bin(hipStream_t st, GridBwdBufs& w, uint32_t B, const float* pos, uint32_t pstride, const void* dy,
                                    int layout, uint32_t dy_stride) const {
	if (bin_levels.empty() || B == 0) return;
	const GridBinArgs a = bin_args(w, B);
	launch_grid_bin(st, desc.n_pos_dims, desc.n_features_per_level, desc.hash_type, B, pos, pstride, dy, layout, dy_stride, dev_levels(),
	                hash_grid(), desc.interp, a, opts());
}

void GridEncodingHost::backward_acc(hipStream_t st, GridBwdBufs& w, uint32_t B, const void* dy, int layout, uint32_t dy_stride,
                                    float* grad32, const GridAccAdam* adam) const {
	if (bin_levels.empty()) return;
	if (B == 0) {  // no points: zero gradient (Overwrite)
		if (!adam) TCNN_HIP_CHECK(hipMemsetAsync(grad32 + n_lds_params, 0, (size_t)(n_params - n_lds_params) * 4, st));
		return;
	}
	const GridBinArgs a = bin_args(w, B);
	launch_grid_acc(st, desc.n_pos_dims, desc.n_features_per_level, B, dy, layout, dy_stride, dev_levels(), a, grad32, adam);
}

void GridEncodingHost::reduce_items(hipStream_t st, GridBwdBufs& w, float* grad32, GradFinalize fin) const {
	if (plans[0].slices.empty()) return;
	launch_grid_slab_reduce(st, w.partial.as<float>(), w.n_chunks, n_lds_params, n_lds_params, grad32, slab_map(w.plan), fin);
}

void GridEncodingHost::backward(hipStream_t st, GridBwdBufs& w, uint32_t B, const float* pos, uint32_t pstride, const void* dy,
                                int layout, uint32_t dy_stride, float* grad32) const {
	backward_items(st, w, B, pos, pstride, dy, layout, dy_stride);
	backward_bin(st, w, B, pos, pstride, dy, layout, dy_stride);
	backward_acc(st, w, B, dy, layout, dy_stride, grad32);
	reduce_items(st, w, grad32);
}

static const char* grid_type_str(GridType t) { return t == GridType::Hash ? "Hash" : t == GridType::Dense ? "Dense" : "Tiled"; }
static const char* hash_str(HashType t) { return t == HashType::Prime ? "Prime" : t == HashType::ReversedPrime ? "ReversedPrime" : "CoherentPrime"; }
static const char* interp_str(Interp t) { return t == Interp::Nearest ? "Nearest" : t == Interp::Smoothstep ? "Smoothstep" : "Linear"; }

json GridEncodingHost::hyperparams() const {  // grid.h:1096-1114
	json r = {
		{"otype", "Grid"}, {"type", grid_type_str(desc.grid_type)}, {"n_levels", desc.n_levels},
		{"n_features_per_level", desc.n_features_per_level}, {"base_resolution", desc.base_resolution},
		{"per_level_scale", desc.per_level_scale}, {"interpolation", interp_str(desc.interp)}, {"hash", hash_str(desc.hash_type)},
	};
	if (desc.grid_type == GridType::Hash) r["log2_hashmap_size"] = desc.log2_hashmap_size;
	return r;
}

// ------------------------------------------------------------------------------------------
// MLP (reference src/network.cu:48-138, fully_fused_mlp.cu:635-678, 865-891)
// ------------------------------------------------------------------------------------------
static const char* const ACT_NAMES[] = {"None", "ReLU", "LeakyReLU", "Exponential", "Sine", "Sigmoid", "Squareplus", "Softplus", "Tanh"};

static int parse_activation(const std::string& s) {  // string_to_activation (common.cu)
	for (int a = 0; a <= ACT_TANH; ++a)
		if (ieq(s, ACT_NAMES[a])) return a;
	throw std::runtime_error("Invalid activation name: " + s);
}

MlpHost::MlpHost(uint32_t n_input_dims, uint32_t n_output_dims, const json& net) {
	otype = jval<std::string>(net, "otype", "MLP");
	TCNN_CHECK(ieq(otype, "FullyFusedMLP") || ieq(otype, "MegakernelMLP") || ieq(otype, "MLP") || ieq(otype, "CutlassMLP"),
	           "Invalid network type: " + otype);
	width = jval<uint32_t>(net, "n_neurons", 128u);
	n_hidden_layers = jval<uint32_t>(net, "n_hidden_layers", 5u);
	if (ieq(otype, "FullyFusedMLP") || ieq(otype, "MegakernelMLP")) {
		TCNN_CHECK(n_hidden_layers >= 1, "FullyFusedMLP requires at least 1 hidden layer (3 layers in total).");
		TCNN_CHECK(width == 16 || width == 32 || width == 64 || width == 128,
		           "FullyFusedMLP only supports 16, 32, 64, and 128 neurons, but got " + std::to_string(width) + ". Use CutlassMLP instead if this is a requirement.");
	}
	// CutlassMLP (cutlass_mlp.cu:41-81): any width; 0 hidden layers = one [padded_output][input] matrix
	activation = parse_activation(jval<std::string>(net, "activation", "ReLU"));
	output_activation = parse_activation(jval<std::string>(net, "output_activation", "None"));
	n_input = n_input_dims;
	n_output = n_output_dims;
	padded_output = (n_output + 15) / 16 * 16;  // REQUIRED_ALIGNMENT 16 (fully_fused_mlp.h:108-110)
}

static void xavier(Pcg32& rnd, uint32_t rows, uint32_t cols, float* out, float scale) {
	scale *= std::sqrt(6.0f / (float)(cols + rows));
	const size_t n = (size_t)rows * cols;
	for (size_t i = 0; i < n; ++i) {
		float t = rnd.next_float() * 2.0f;
		t = t * scale;
		out[i] = t - scale;
	}
}

void MlpHost::initialize_params(Pcg32& rng, float* out, float scale) const {
	if (n_hidden_layers == 0) {  // one matrix (cutlass_mlp.cu:64-67)
		xavier(rng, padded_output, n_input, out, scale);
		return;
	}
	xavier(rng, width, n_input, out, scale);
	out += (size_t)width * n_input;
	for (uint32_t i = 1; i < n_hidden_layers; ++i) {
		xavier(rng, width, width, out, scale);
		out += (size_t)width * width;
	}
	xavier(rng, padded_output, width, out, scale);
}

static const char* act_str(int a) { return a >= 0 && a <= ACT_TANH ? ACT_NAMES[a] : "None"; }

json MlpHost::hyperparams() const {
	return {{"otype", ieq(otype, "CutlassMLP") || ieq(otype, "MLP") ? "CutlassMLP" : "FullyFusedMLP"},
	        {"n_neurons", width}, {"n_hidden_layers", n_hidden_layers},
	        {"activation", act_str(activation)}, {"output_activation", act_str(output_activation)}};
}

void AdamHost::update(const json& p) {  // adam.h:235-283
	if (jhas(p, "beta1")) beta1 = p["beta1"].get<float>();
	if (jhas(p, "beta2")) beta2 = p["beta2"].get<float>();
	if (jhas(p, "epsilon")) epsilon = p["epsilon"].get<float>();
	if (jhas(p, "learning_rate")) learning_rate = p["learning_rate"].get<float>();
	if (jhas(p, "l2_reg")) l2_reg = p["l2_reg"].get<float>();
	if (jhas(p, "adabound")) adabound = p["adabound"].get<bool>();
	if (jhas(p, "relative_decay")) relative_decay = p["relative_decay"].get<float>();
	if (jhas(p, "absolute_decay")) absolute_decay = p["absolute_decay"].get<float>();
	if (jhas(p, "clipping_magnitude")) clipping_magnitude = p["clipping_magnitude"].get<float>();
	if (jhas(p, "non_matrix_learning_rate_factor")) non_matrix_learning_rate_factor = p["non_matrix_learning_rate_factor"].get<float>();
	if (jhas(p, "optimize_matrix_params")) optimize_matrix_params = p["optimize_matrix_params"].get<bool>();
	if (jhas(p, "optimize_non_matrix_params")) optimize_non_matrix_params = p["optimize_non_matrix_params"].get<bool>();
}

json AdamHost::hyperparams() const {
	return {{"otype", "Adam"}, {"beta1", beta1}, {"beta2", beta2}, {"epsilon", epsilon}, {"learning_rate", learning_rate},
	        {"l2_reg", l2_reg}, {"adabound", adabound}, {"relative_decay", relative_decay}, {"absolute_decay", absolute_decay},
	        {"clipping_magnitude", clipping_magnitude}, {"non_matrix_learning_rate_factor", non_matrix_learning_rate_factor},
	        {"optimize_matrix_params", optimize_matrix_params}, {"optimize_non_matrix_params", optimize_non_matrix_params}};
}

// ------------------------------------------------------------------------------------------
// Encodings (reference src/encoding.cu:77-150)
// ------------------------------------------------------------------------------------------
bool EncodingHost::known(const std::string& eo) {
	return ieq(eo, "HashGrid") || ieq(eo, "Grid") || ieq(eo, "TiledGrid") || ieq(eo, "DenseGrid") || ieq(eo, "OneBlob") ||
	       ieq(eo, "Identity");
}

EncodingHost::EncodingHost(uint32_t n_dims_to_encode, const json& enc) : n_dims(n_dims_to_encode) {
	const std::string eo = jval<std::string>(enc, "otype", "OneBlob");  // encoding.cu:133
	TCNN_CHECK(known(eo), "Encoding '" + eo + "' is not implemented by the MI355X engine yet");
	if (ieq(eo, "OneBlob")) {
		kind = EncKind::OneBlob;
		n_bins = jval<uint32_t>(enc, "n_bins", 16u);  // encoding.cu:81-83
		TCNN_CHECK(n_bins > 0 && (n_bins & (n_bins - 1)) == 0, "Number of bins must be a power of 2");
	} else if (ieq(eo, "Identity")) {
		kind = EncKind::Identity;
		scale = jval<float>(enc, "scale", 1.0f);  // encoding.cu:77-79
		offset = jval<float>(enc, "offset", 0.0f);
	} else {
		kind = EncKind::Grid;
		grid = std::make_unique<GridEncodingHost>(n_dims_to_encode, enc);
	}
}

uint32_t EncodingHost::n_output_unpadded() const {
	switch (kind) {
		case EncKind::OneBlob: return n_dims * n_bins;
		case EncKind::Identity: return n_dims;
		default: return grid->n_features;
	}
}

void EncodingHost::set_alignment(uint32_t a) {  // Encoding::set_alignment (encoding.h)
	if (kind == EncKind::Grid) {
		grid->set_alignment(a);
		return;
	}
	const uint32_t n = n_output_unpadded();
	n_to_pad = (n + a - 1) / a * a - n;
}

void EncodingHost::initialize_params(Pcg32& rng, float* out, float s) const {
	if (kind == EncKind::Grid) grid->initialize_params(rng, out, s);
}

json EncodingHost::hyperparams() const {
	switch (kind) {
		case EncKind::OneBlob: return {{"otype", "OneBlob"}, {"n_bins", n_bins}};
		case EncKind::Identity: return {{"otype", "Identity"}, {"scale", scale}, {"offset", offset}};
		default: return grid->hyperparams();
	}
}

void EncodingHost::forward_aos(hipStream_t st, uint32_t B, const float* x, const void* params16, void* out16) const {
	const uint32_t W = padded_output_width();
	switch (kind) {
		case EncKind::OneBlob: launch_oneblob_fwd(st, B, n_dims, n_bins, x, n_dims, out16, W, n_to_pad); break;
		case EncKind::Identity: launch_identity_fwd(st, B, n_dims, scale, offset, x, n_dims, out16, W, n_to_pad); break;
		default:
			if (grid->n_to_pad) TCNN_HIP_CHECK(hipMemsetAsync(out16, 0, (size_t)B * W * 2, st));
			launch_grid_fwd(st, grid->desc.n_pos_dims, grid->desc.n_features_per_level, grid->desc.hash_type, B, grid->desc.n_levels, x,
			                grid->desc.n_pos_dims, params16, out16, false, W, grid->dev_levels(), grid->hash_grid(), grid->desc.interp,
			                grid->opts());
	}
}

void EncodingHost::backward_input(hipStream_t st, uint32_t B, const float* x, const void* dy16, float* dx, const void* params16,
                                  int dy_layout) const {
	const uint32_t W = padded_output_width();
	switch (kind) {
		case EncKind::OneBlob: launch_oneblob_bwd(st, B, n_dims, n_bins, x, n_dims, dy16, W, dx, n_dims); break;
		case EncKind::Identity: launch_identity_bwd(st, B, n_dims, scale, dy16, W, dx, n_dims); break;
		default:
			TCNN_CHECK(params16, "grid backward_input needs the grid parameters");
			launch_grid_bwd_input(st, grid->desc.n_pos_dims, grid->desc.n_features_per_level, grid->desc.hash_type, B, grid->desc.n_levels,
			                      x, grid->desc.n_pos_dims, params16, dy16, dy_layout, W, dx, n_dims, grid->dev_levels(), grid->hash_grid(),
			                      grid->desc.interp, grid->opts());
	}
}

// ------------------------------------------------------------------------------------------
// NetworkWithInputEncoding
// ------------------------------------------------------------------------------------------
NetworkHost::NetworkHost(uint32_t n_in, uint32_t n_out, const json& e, const json& net) : n_input_dims(n_in), n_output_dims(n_out) {
	enc = std::make_unique<EncodingHost>(n_in, e);
	grid = enc->grid.get();
	enc->set_alignment(16);  // minimum_alignment(network): 16 for FullyFusedMLP and CutlassMLP (network.cu:76-95)
	mlp = MlpHost(enc->padded_output_width(), n_out, net);
	TCNN_CHECK(fused_ok() || layered_ok(), "network shape (n_neurons = " + std::to_string(mlp.width) + ", input width " +
	                                           std::to_string(mlp.n_input) + ") is not supported by the MI355X engine");
	log_debug(std::string("NetworkWithInputEncoding: ") + mlp.otype + " (n_neurons=" + std::to_string(mlp.width) +
	          ", n_hidden_layers=" + std::to_string(mlp.n_hidden_layers) + ") runs on the " + engine() + " engine");
}

bool NetworkHost::fused_ok() const {
	// CutlassMLP / "MLP" run on the layer-wise engine (the reference's separate GEMM-per-layer network)
	const bool ff = ieq(mlp.otype, "FullyFusedMLP") || ieq(mlp.otype, "MegakernelMLP");
	if (sw.no_fused_grid) return false;  // A/B switch: the tile engine instead
	return ff && grid && grid->n_to_pad == 0 && !grid->opts().active && mlp.output_activation == 0 &&
	       (mlp.activation == ACT_NONE || mlp.activation == ACT_RELU) &&
	       fused_train_supported(mlp.width, mlp.n_input, mlp.n_hidden_layers, grid->desc.n_pos_dims,
	                             grid->desc.n_features_per_level, mlp.padded_output, mlp.activation, grid->desc.hash_type);
}

bool NetworkHost::tile_shape_ok() const {
	const bool ff = ieq(mlp.otype, "FullyFusedMLP") || ieq(mlp.otype, "MegakernelMLP");
	if (!ff || mlp.output_activation == ACT_SINE) return false;  // Sine has no post-activation backward (common_device.h:271-275)
	if (sw.no_tile_engine) return false;  // A/B switch: the layer-wise engine instead
	return tile_train_supported(mlp.width, mlp.n_input, mlp.n_hidden_layers, mlp.padded_output, mlp.activation);
}

bool NetworkHost::tile_ok() const { return !fused_ok() && tile_shape_ok(); }

bool NetworkHost::tile_infer_ok() const {
	return tile_shape_ok() && tile_infer_supported(mlp.width, mlp.n_input, mlp.n_hidden_layers, mlp.padded_output, mlp.activation);
}

const char* NetworkHost::inference_engine() const {
	if (fused_ok() && mlp_infer_supported(mlp.width, mlp.n_input, mlp.n_hidden_layers, mlp.padded_output, mlp.activation)) return "fused";
	if (tile_infer_ok()) return "fused";
	return layered_ok() ? "layered" : "unsupported";
}

// any width / input width / padded output that is a multiple of 16 (layers above 128 run k_wide_layer)
bool NetworkHost::layered_ok() const {
	return layered_width_supported(mlp.width) && mlp.n_input % 16 == 0 && layered_width_supported(mlp.n_input) &&
	       layered_width_supported(mlp.padded_output) && mlp.activation != ACT_SINE &&
	       mlp.output_activation != ACT_SINE;  // Sine has no post-activation backward
}

void NetworkHost::initialize_params(Pcg32& rng, float* out, float scale) const {
	mlp.initialize_params(rng, out, scale);
	enc->initialize_params(rng, out + mlp.n_params(), scale);
}

json NetworkHost::hyperparams() const {
	return {{"otype", "NetworkWithInputEncoding"}, {"encoding", enc->hyperparams()}, {"network", mlp.hyperparams()}};
}

void NetworkHost::forward_layers(hipStream_t st, StepWorkspace& ws, uint32_t B, const void* params16, void* out16, bool keep) {
	const uint32_t W = mlp.width, IN = mlp.n_input, NH = mlp.n_hidden_layers, OUTP = mlp.padded_output;
	const _Float16* p = (const _Float16*)params16;
	ws.acts.reserve((size_t)(keep ? NH : 2) * B * W * 2);
	auto act_buf = [&](uint32_t j) { return ws.acts.as<_Float16>() + (size_t)(keep ? j : (j & 1)) * B * W; };
	const void* x = ws.enc16.p;
	uint32_t K = IN;
	for (uint32_t j = 0; j < NH; ++j) {
		launch_layer_fwd(st, B, W, K, p, x, act_buf(j), mlp.activation);
		p += (size_t)W * K;
		x = act_buf(j);
		K = W;
	}
	launch_layer_fwd(st, B, OUTP, K, p, x, out16, mlp.output_activation);
}

void NetworkHost::inference(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const void* params16, void* out16,
                            bool trust_image) {
	TCNN_CHECK(B % 32 == 0, "inference: batch must be a multiple of 32");
	const uint32_t IN = mlp.n_input;
	const uint8_t* eparams = (const uint8_t*)params16 + (size_t)mlp.n_params() * 2;
	if (fused_ok() && mlp_infer_supported(mlp.width, IN, mlp.n_hidden_layers, mlp.padded_output, mlp.activation)) {
		// the trainer's packed image when it matches its parameters, else the kernel builds its LDS
		// image from the parameters themselves (no pack launch)
		fused_forward(st, ws, B, pos, params16, trust_image && ws.wimage_valid, nullptr, out16);
		return;
	}
	ws.enc16.reserve((size_t)IN * B * 2);
	if (tile_infer_ok()) {  // the whole network in one launch (mlp_tile.h k_mlp_tile_infer)
		enc->forward_aos(st, B, pos, eparams, ws.enc16.p);
		launch_mlp_tile_infer(st, mlp.width, IN, mlp.n_hidden_layers, mlp.activation, mlp.output_activation, B, params16, ws.enc16.p, out16);
		return;
	}
	TCNN_CHECK(layered_ok(), "inference: network shape not supported by the MI355X engine");
	enc->forward_aos(st, B, pos, eparams, ws.enc16.p);
	forward_layers(st, ws, B, params16, out16, false);
}

// grid encoding + MLP forward on the packed weight image (ws.wimage): one kernel (k_fused_fwd_grid),
// or under TCNN_SPLIT_FORWARD the SoA grid forward then k_mlp_infer. enc_soa (nullable) receives the
// encoding [IN][B] for a training context's backward.
void NetworkHost::fused_forward(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const void* params16, bool use_image,
                                void* enc_soa, void* out16) {
	const uint32_t IN = mlp.n_input;
	const uint8_t* eparams = (const uint8_t*)params16 + (size_t)mlp.n_params() * 2;
	if (sw.split_forward) {
		if (!use_image) {
			ws.wimage.reserve(fused_weight_image_bytes(mlp.width, IN, mlp.n_hidden_layers));
			launch_pack_weights(st, mlp.width, IN, mlp.n_hidden_layers, params16, ws.wimage.p);
			ws.wimage_valid = false;  // packed from these parameters, which need not be the trainer's
		}
		void* enc = enc_soa;
		if (!enc) {
			ws.enc16.reserve((size_t)IN * B * 2);
			enc = ws.enc16.p;
		}
		launch_grid_fwd(st, grid->desc.n_pos_dims, grid->desc.n_features_per_level, grid->desc.hash_type, B, grid->desc.n_levels, pos,
		                grid->desc.n_pos_dims, eparams, enc, true, 0, grid->dev_levels(), grid->hash_grid(), grid->desc.interp,
		                grid->opts());
		launch_mlp_infer(st, mlp.width, IN, mlp.n_hidden_layers, mlp.activation, true, B, ws.wimage.p, enc, out16);
		return;
	}
	if (!use_image && ((uintptr_t)params16 & 15)) {
		// the kernel builds its LDS image with 16-byte loads from aligned parameters; a parameter view
		// with an odd offset (e.g. a slice of a flat torch buffer) gets the packed image instead
		ws.wimage.reserve(fused_weight_image_bytes(mlp.width, IN, mlp.n_hidden_layers));
		launch_pack_weights(st, mlp.width, IN, mlp.n_hidden_layers, params16, ws.wimage.p);
		ws.wimage_valid = false;  // packed from these parameters, which need not be the trainer's
		use_image = true;
	}
	launch_fused_fwd(st, mlp.width, IN, mlp.n_hidden_layers, grid->desc.n_pos_dims, grid->desc.hash_type, mlp.activation, B,
	                 use_image ? ws.wimage.p : nullptr, params16, eparams, pos, grid->dev_levels(), grid->hash_grid(), grid->desc.interp,
	                 grid->inrange_index_ok && grid->desc.interp == Interp::Linear && !sw.no_inrange_index, enc_soa, out16);
}

int NetworkHost::backward_engine_keep(bool with_dinput) const {
	if (fused_ok() && !with_dinput) return KEEP_FUSED_SOA;
	if (tile_shape_ok()) return KEEP_TILE_AOS;
	return KEEP_NONE;
}

int NetworkHost::forward_keep(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const void* params16, void* out16,
                              bool with_dinput, DevBuf& keep) {
	const int layout = backward_engine_keep(with_dinput);
	const uint32_t IN = mlp.n_input;
	const uint8_t* eparams = (const uint8_t*)params16 + (size_t)mlp.n_params() * 2;
	if (layout == KEEP_FUSED_SOA && mlp_infer_supported(mlp.width, IN, mlp.n_hidden_layers, mlp.padded_output, mlp.activation)) {
		keep.reserve((size_t)IN * B * 2);
		fused_forward(st, ws, B, pos, params16, false, keep.p, out16);
		return KEEP_FUSED_SOA;
	}
	if (layout == KEEP_TILE_AOS && tile_infer_ok()) {
		keep.reserve((size_t)IN * B * 2);
		enc->forward_aos(st, B, pos, eparams, keep.p);
		launch_mlp_tile_infer(st, mlp.width, IN, mlp.n_hidden_layers, mlp.activation, mlp.output_activation, B, params16, keep.p, out16);
		return KEEP_TILE_AOS;
	}
	inference(st, ws, B, pos, params16, out16);
	return KEEP_NONE;
}

void NetworkHost::fwd_bwd(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const float* target, uint32_t dims,
                          float loss_scale, const void* params16, const void* dout16, void* out16, float* grad32,
                          const std::function<void(int)>& mark, float* dL_dinput, const void* kept, int kept_layout) {
	if (fused_ok() && !dL_dinput)
		fwd_bwd_fused(st, ws, B, pos, target, dims, loss_scale, params16, dout16, out16, grad32, mark,
		              kept_layout == KEEP_FUSED_SOA ? kept : nullptr);
	else if (tile_shape_ok())
		fwd_bwd_tile(st, ws, B, pos, target, dims, loss_scale, params16, dout16, out16, grad32, mark, dL_dinput,
		             kept_layout == KEEP_TILE_AOS ? kept : nullptr);
	else fwd_bwd_layered(st, ws, B, pos, target, dims, loss_scale, params16, dout16, out16, grad32, mark, dL_dinput);
}

void NetworkHost::pack_weights(hipStream_t st, StepWorkspace& ws, const void* params16) {
	ws.wimage.reserve(fused_weight_image_bytes(mlp.width, mlp.n_input, mlp.n_hidden_layers));
	launch_pack_weights(st, mlp.width, mlp.n_input, mlp.n_hidden_layers, params16, ws.wimage.p);
	ws.wimage_valid = true;
}

void NetworkHost::fused_kernel(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const float* target, uint32_t dims,
                               float loss_scale, const void* params16, bool pack, const void* dout16, void* out16, const void* enc_soa) {
	TCNN_CHECK(B % 32 == 0, "training: batch must be a multiple of 32");
	const uint32_t n_mlp = mlp.n_params();
	const uint32_t L = grid->desc.n_levels, F = grid->desc.n_features_per_level;
	const uint32_t nb = fused_train_n_blocks(mlp.width, mlp.n_input, mlp.n_hidden_layers, grid->desc.n_pos_dims, dims,
	                                         dout16 != nullptr, B);
	ws.n_fused_blocks = nb;
	ws.n_loss_partials = nb;
	ws.dLdenc.reserve((size_t)L * F * B * 2);
	ws.wgrad_partial.reserve((size_t)nb * n_mlp * 4);
	ws.loss_partial.reserve((size_t)nb * 4);
	// without a packed image that matches params16, every workgroup builds its LDS image from the
	// parameters (load_weights_lds_v) -- no k_pack_weights launch; the Adam tail of the grid backward
	// still writes the next step's image into ws.wimage
	ws.wimage.reserve(fused_weight_image_bytes(mlp.width, mlp.n_input, mlp.n_hidden_layers));
	bool use_image = !pack && ws.wimage_valid;
	if (!use_image && ((uintptr_t)params16 & 15)) {  // unaligned parameter view: pack the image (see fused_forward)
		launch_pack_weights(st, mlp.width, mlp.n_input, mlp.n_hidden_layers, params16, ws.wimage.p);
		ws.wimage_valid = false;
		use_image = true;
	}
	const uint8_t* table = (const uint8_t*)params16 + (size_t)n_mlp * 2;
	launch_fused_train(st, mlp.width, mlp.n_input, mlp.n_hidden_layers, grid->desc.n_pos_dims, grid->desc.hash_type,
	                   mlp.activation, B, dims, loss_scale, params16, table, pos, target, out16, ws.dLdenc.p,
	                   ws.wgrad_partial.as<float>(), ws.loss_partial.as<float>(), grid->dev_levels(), grid->hash_grid(),
	                   grid->desc.interp, nb, dout16, use_image ? ws.wimage.p : nullptr, loss_l2,
	                   grid->inrange_index_ok && grid->desc.interp == Interp::Linear && !sw.no_inrange_index, enc_soa,
	                   dout16 ? ext_dout_scale : 1.0f);
}

void NetworkHost::grid_backward(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, GridBwdEpilogue* ep) {
	if (ep) {
		ep->wimage = ws.wimage.as<_Float16>();
		ep->W = mlp.width;
		ep->IN = mlp.n_input;
		ep->NH = mlp.n_hidden_layers;
		fused_image_layout(mlp.width, mlp.n_input, mlp.n_hidden_layers, &ep->RSI, &ep->RSW, &ep->oWh, &ep->oWo);
		ep->wpart = ws.wgrad_partial.as<float>();
		ep->n_wparts = ws.n_fused_blocks;
		ep->lpart = ws.loss_partial.as<float>();
	}
	grid->backward_items(st, ws.gbw, B, pos, grid->desc.n_pos_dims, ws.dLdenc.p, 0, 0, ep, ep ? ep->n_mlp_groups : 0u);
	grid->backward_bin(st, ws.gbw, B, pos, grid->desc.n_pos_dims, ws.dLdenc.p, 0, 0);
	if (ep && ep->apply_adam) ws.wimage_valid = true;  // the epilogue wrote the image of the updated weights
}

void NetworkHost::fwd_bwd_fused(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const float* target,
                                uint32_t dims, float loss_scale, const void* params16, const void* dout16, void* out16, float* grad32,
                                const std::function<void(int)>& mark, const void* enc_soa) {
	const uint32_t n_mlp = mlp.n_params();
	fused_kernel(st, ws, B, pos, target, dims, loss_scale, params16, true, dout16, out16, enc_soa);
	if (mark) mark(1);
	// the network-gradient column sums run in the grid backward's spare workgroups (the epilogue
	// without Adam: block_column_sums, the order of launch_column_sums), not as a launch of their own
	GridBwdEpilogue ep{};
	ep.enabled = 1;
	ep.apply_adam = 0;
	ep.buf.g32 = grad32;
	ep.n_mlp_groups = mlp_tail_groups();
	ep.n_mlp = n_mlp;
	ws.loss_sum.reserve(16);
	ep.d_loss = ws.loss_sum.as<float>();
	TCNN_CHECK(n_mlp % 4 == 0, "network parameter count must be a multiple of 4");
	// the torch binding's finalised gradient straight from the two reductions (no k_grad_finalize
	// pass) when every grid level goes through the slabs
	const bool fin = grad_fin.out && grid->bin_levels.empty();
	GradFinalize fin_grid{};
	if (fin) {
		ep.fin = grad_fin;
		fin_grid = grad_fin;
		fin_grid.out = (char*)grad_fin.out + (size_t)n_mlp * (grad_fin.out_f32 ? 4 : 2);
	}
	grad_fin_done = fin;
	grid_backward(st, ws, B, pos, &ep);
	grid->backward_acc(st, ws.gbw, B, ws.dLdenc.p, 0, 0, grad32 + n_mlp);
	if (mark) mark(2);
	grid->reduce_items(st, ws.gbw, grad32 + n_mlp, fin_grid);
	if (mark) mark(3);
}

// Tile-engine training pass (mlp_tile.hip): encoding forward (AoS fp16), one fused kernel for the
// whole network over 32-sample tiles (forward, loss, backward, weight-gradient partials, dL/d(enc)),
// the partial reduction, then the encoding's backward.
void NetworkHost::fwd_bwd_tile(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const float* target, uint32_t dims,
                               float loss_scale, const void* params16, const void* dout16, void* out16, float* grad32,
                               const std::function<void(int)>& mark, float* dL_dinput, const void* enc_aos) {
	TCNN_CHECK(B % 32 == 0, "training: batch must be a multiple of 32");
	const uint32_t W = mlp.width, IN = mlp.n_input, NH = mlp.n_hidden_layers;
	const uint32_t n_mlp = mlp.n_params();
	const uint8_t* eparams = (const uint8_t*)params16 + (size_t)n_mlp * 2;
	// configs[3]-shaped networks gather the grid encoding inside the tile kernel (no AoS pass)
	TileGridEnc genc{};
	const bool in_kernel = !enc_aos && grid && grid->desc.n_pos_dims == 2 && grid->desc.n_features_per_level == 2 &&
	                       grid->n_to_pad == 0 && grid->desc.interp == Interp::Linear && !grid->opts().active &&
	                       tile_train_genc_ok(W, IN, NH, mlp.activation, B, grid->desc.hash_type);
	if (in_kernel) {
		genc.pos = pos;
		genc.table16 = eparams;
		genc.levels = grid->dev_levels();
		genc.hash = grid->desc.hash_type;
		genc.hash_grid = grid->hash_grid() ? 1u : 0u;
		genc.inrange = grid->opts().inrange_index;
	} else if (!enc_aos) {
		ws.enc16.reserve((size_t)B * IN * 2);
		enc->forward_aos(st, B, pos, eparams, ws.enc16.p);
		enc_aos = ws.enc16.p;
	}
	const uint32_t nb = tile_train_blocks(B, W, IN, NH);
	ws.wgrad_partial.reserve((size_t)nb * n_mlp * 4);
	ws.loss_partial.reserve((size_t)nb * 4);
	const bool enc_grad = enc->n_params() > 0 || dL_dinput;
	// a grid with feature pairs and no padding takes dL/d(encoding) as level-major pairs [L][B]
	const bool pairs = grid && grid->desc.n_features_per_level == 2 && grid->n_to_pad == 0;
	if (enc_grad) ws.delta0.reserve((size_t)B * IN * 2);
	const uint32_t wT_bytes = tile_train_wT_bytes(W, IN, NH);
	if (wT_bytes) ws.tile_wT.reserve(wT_bytes);
	launch_mlp_tile_train(st, W, IN, NH, mlp.activation, mlp.output_activation, B, dims, loss_scale, loss_l2, params16, enc_aos, target,
	                      dout16, out16,
	                      enc_grad ? ws.delta0.p : nullptr, pairs ? 1 : 0, ws.wgrad_partial.as<float>(), ws.loss_partial.as<float>(),
	                      wT_bytes ? ws.tile_wT.p : nullptr, in_kernel ? &genc : nullptr);
	ws.n_loss_partials = dout16 ? 0 : nb;
	const size_t tf = reduce_partials_tmp_floats(nb, n_mlp);
	if (tf) ws.red_tmp.reserve(tf * 4);
	launch_reduce_partials(st, ws.wgrad_partial.as<float>(), nb, n_mlp, n_mlp, grad32, ws.red_tmp.as<float>());
	if (mark) mark(1);
	const int dy_layout = pairs ? 0 : 2;
	if (dL_dinput) enc->backward_input(st, B, pos, ws.delta0.p, dL_dinput, eparams, dy_layout);
	if (grid) grid->backward(st, ws.gbw, B, pos, grid->desc.n_pos_dims, ws.delta0.p, dy_layout, IN, grad32 + n_mlp);
	if (mark) mark(2);
	if (mark) mark(3);
}

// Layer-wise training pass (reference FullyFusedMLP::forward_impl/backward_impl dataflow,
// fully_fused_mlp.cu:680-836; CutlassMLP cutlass_mlp.cu:120-315).
void NetworkHost::fwd_bwd_layered(hipStream_t st, StepWorkspace& ws, uint32_t B, const float* pos, const float* target,
                                  uint32_t dims, float loss_scale, const void* params16, const void* dout16, void* out16,
                                  float* grad32, const std::function<void(int)>& mark, float* dL_dinput) {
	TCNN_CHECK(layered_ok(), "training: network/encoding configuration not supported by the MI355X engine");
	TCNN_CHECK(B % 32 == 0, "training: batch must be a multiple of 32");
	const uint32_t W = mlp.width, IN = mlp.n_input, NH = mlp.n_hidden_layers, OUTP = mlp.padded_output;
	const uint32_t n_mlp = mlp.n_params();
	const _Float16* p16 = (const _Float16*)params16;
	const uint8_t* eparams = (const uint8_t*)params16 + (size_t)n_mlp * 2;
	const uint32_t nck = wgrad_n_chunks(B);
	const uint32_t maxK = std::max(W, IN);
	ws.enc16.reserve((size_t)B * IN * 2);
	ws.out16.reserve((size_t)B * OUTP * 2);
	ws.dout16.reserve((size_t)B * OUTP * 2);
	ws.delta0.reserve((size_t)B * std::max(W, IN) * 2);
	ws.delta1.reserve((size_t)B * std::max(W, IN) * 2);
	ws.wgrad_partial.reserve((size_t)nck * std::max(W, OUTP) * maxK * 4);

	// forward
	enc->forward_aos(st, B, pos, eparams, ws.enc16.p);
	void* out = out16 ? out16 : ws.out16.p;
	forward_layers(st, ws, B, params16, out, true);
	auto act = [&](uint32_t j) { return ws.acts.as<_Float16>() + (size_t)j * B * W; };

	// loss / external dL/dout (loss-scaled by the caller) -> G fp16 [B][OUTP]
	if (dout16) {
		TCNN_HIP_CHECK(hipMemcpyAsync(ws.dout16.p, dout16, (size_t)B * OUTP * 2, hipMemcpyDeviceToDevice, st));
		ws.n_loss_partials = 0;
	} else {
		const uint32_t nl = relative_l2_n_blocks(B, OUTP);
		ws.loss_partial.reserve((size_t)nl * 4);
		launch_relative_l2_partial(st, B, OUTP, dims, loss_scale, out, target, ws.dout16.p, ws.loss_partial.as<float>(), loss_l2);
		ws.n_loss_partials = nl;
	}
	launch_act_bwd_inplace(st, B * OUTP, mlp.output_activation, out, ws.dout16.p);

	// backward: weight offsets [W0 | W1..W_{NH-1} | Wout] ([Wout] alone for 0 hidden layers)
	auto w_off = [&](uint32_t j) -> size_t { return j == 0 ? 0 : (size_t)W * IN + (size_t)(j - 1) * W * W; };
	auto wgrad = [&](uint32_t N, uint32_t K, const void* dy, const void* x, size_t off) {
		launch_wgrad(st, B, N, K, dy, x, ws.wgrad_partial.as<float>(), nck);
		const size_t tf = reduce_partials_tmp_floats(nck, N * K);
		if (tf) ws.red_tmp.reserve(tf * 4);
		launch_reduce_partials(st, ws.wgrad_partial.as<float>(), nck, N * K, N * K, grad32 + off, ws.red_tmp.as<float>());
	};
	_Float16* dcur = ws.delta0.as<_Float16>();
	_Float16* dnext = ws.delta1.as<_Float16>();
	const bool enc_grad = enc->n_params() > 0 || dL_dinput;
	// a grid with feature pairs and no padding takes dL/d(encoding) as level-major pairs [L][B], the
	// layout its backward reads coalesced (AoS rows would cost one 64-byte line per 4-byte read)
	const bool pairs = grid && grid->desc.n_features_per_level == 2 && grid->n_to_pad == 0;
	const int dy_layout = pairs ? 0 : 2;
	const _Float16* denc = dnext;  // dL/d(encoding), when enc_grad
	if (NH == 0) {  // one matrix: dWout = dout^T enc, dL/d(encoding) = Wout^T dout (no transfer)
		wgrad(OUTP, IN, ws.dout16.p, ws.enc16.p, 0);
		if (mark) mark(1);
		if (enc_grad) launch_layer_bwd(st, B, OUTP, IN, p16, ws.dout16.p, nullptr, dnext, ACT_NONE, pairs);
	} else {
		// output layer
		wgrad(OUTP, W, ws.dout16.p, act(NH - 1), w_off(NH));
		launch_layer_bwd(st, B, OUTP, W, p16 + w_off(NH), ws.dout16.p, act(NH - 1), dcur, mlp.activation);
		for (uint32_t j = NH - 1; j >= 1; --j) {
			wgrad(W, W, dcur, act(j - 1), w_off(j));
			launch_layer_bwd(st, B, W, W, p16 + w_off(j), dcur, act(j - 1), dnext, mlp.activation);
			std::swap(dcur, dnext);
		}
		wgrad(W, IN, dcur, ws.enc16.p, 0);
		if (mark) mark(1);
		// dL/d(encoding) = W0^T delta_0 (no transfer), AoS [B][IN] or level-major pairs
		if (enc_grad) launch_layer_bwd(st, B, W, IN, p16, dcur, nullptr, dnext, ACT_NONE, pairs);
		denc = dnext;
	}
	if (enc_grad && dL_dinput) enc->backward_input(st, B, pos, denc, dL_dinput, eparams, dy_layout);
	if (grid) {
		grid->backward(st, ws.gbw, B, pos, grid->desc.n_pos_dims, denc, dy_layout, IN, grad32 + n_mlp);
	}
	if (mark) mark(2);
	if (mark) mark(3);
}

// ------------------------------------------------------------------------------------------
// Trainer (reference trainer.h:47-361, config.h:46-63)
// ------------------------------------------------------------------------------------------
TrainerHost::TrainerHost(uint32_t n_in, uint32_t n_out, const json& cfg, uint32_t seed)
	: n_input_dims(n_in), n_output_dims(n_out), config(cfg) {
	const json enc = jhas(cfg, "encoding") ? cfg["encoding"] : json::object();
	const json net = jhas(cfg, "network") ? cfg["network"] : json::object();
	const json opt = jhas(cfg, "optimizer") ? cfg["optimizer"] : json::object();
	const json los = jhas(cfg, "loss") ? cfg["loss"] : json::object();
	loss_otype = jval<std::string>(los, "otype", "RelativeL2");
	TCNN_CHECK(ieq(loss_otype, "RelativeL2") || ieq(loss_otype, "L2"),
	           "Loss '" + loss_otype + "' is not implemented by the MI355X engine (RelativeL2, L2)");
	const std::string oo = jval<std::string>(opt, "otype", "Adam");
	TCNN_CHECK(ieq(oo, "Adam"), "Optimizer '" + oo + "' is not implemented by the MI355X engine yet");
	adam.update(opt);
	model = std::make_unique<NetworkHost>(n_in, n_out, enc, net);
	model->loss_l2 = ieq(loss_otype, "L2") ? 1u : 0u;
	n_params = model->n_params();
	n_mlp = model->mlp.n_params();
	initialize_params(seed);
}

void TrainerHost::initialize_params(uint32_t seed) {
	// trainer.h:52-55: pcg32{seed_seq{seed}.generate()[0]}
	std::seed_seq seq{seed};
	std::vector<uint32_t> seeds(2);
	seq.generate(seeds.begin(), seeds.end());
	Pcg32 rng{seeds.front()};
	initialize_params_rng(rng);
}

void TrainerHost::initialize_params_rng(Pcg32& rng) {
	log_debug("Trainer: initializing " + std::to_string(n_params) + " params and resetting training.");  // trainer.h:70
	TCNN_HIP_CHECK(hipDeviceSynchronize());  // queued steps on the caller's stream must not race the reset
	std::vector<float> host(n_params);
	model->initialize_params(rng, host.data());
	w32.reserve(n_params * 4);
	w16.reserve(n_params * 2);
	g16.reserve(n_params * 2);
	g32.reserve(n_params * 4);
	m1.reserve(n_params * 4);
	m2.reserve(n_params * 4);
	steps.reserve(n_params * 4);
	d_loss.reserve(16);
	TCNN_HIP_CHECK(hipMemcpy(w32.p, host.data(), n_params * 4, hipMemcpyHostToDevice));
	TCNN_HIP_CHECK(hipMemset(g16.p, 0, n_params * 2));
	TCNN_HIP_CHECK(hipMemset(g32.p, 0, n_params * 4));
	TCNN_HIP_CHECK(hipMemset(m1.p, 0, n_params * 4));
	TCNN_HIP_CHECK(hipMemset(m2.p, 0, n_params * 4));
	TCNN_HIP_CHECK(hipMemset(steps.p, 0, n_params * 4));
	TCNN_HIP_CHECK(hipMemset(d_loss.p, 0, 16));
	launch_cast_f32_f16(nullptr, w32.as<float>(), w16.p, n_params);
	TCNN_HIP_CHECK(hipDeviceSynchronize());
	adam_step = 0;
	ws.wimage_valid = false;
}

void TrainerHost::set_params_full_precision(const float* host, uint64_t n) {
	TCNN_CHECK(n == n_params, "Can't set fp params because buffer has the wrong size.");
	TCNN_HIP_CHECK(hipDeviceSynchronize());  // queued training work must not race the upload
	TCNN_HIP_CHECK(hipMemcpy(w32.p, host, n * 4, hipMemcpyHostToDevice));
	launch_cast_f32_f16(nullptr, w32.as<float>(), w16.p, n_params);
	ws.wimage_valid = false;
	TCNN_HIP_CHECK(hipDeviceSynchronize());
}

void TrainerHost::training_step(hipStream_t st, uint32_t B, const float* input, const float* target, bool run_optimizer) {
	TCNN_CHECK(B % BATCH_GRANULARITY == 0, "training_step: batch size must be a multiple of 256");
	if (timer.enabled) {
		timer.sampling = (timer.counter++ % timer.every) == 0;
		if (timer.sampling) timer.marks.push_back({-1, -1, -1, -1, -1});
	}
	// a whole step with the optimizer replays as a hipGraph when enabled (not on the steps that record
	// phase events, not with AdaBound, whose bounds depend on the step)
	if (run_optimizer && use_graph && !(timer.enabled && timer.sampling) && !adam.adabound && training_step_graph(st, B, input, target))
		return;
	if (run_optimizer) {
		step_eager(st, B, input, target);
		return;
	}
	if (overlapped_ok()) {
		training_step_overlapped(st, B, input, target, false);
		return;
	}
	training_step_sequential(st, B, input, target, false);
}

// the eager step with the optimizer, on whichever schedule is attached
void TrainerHost::step_eager(hipStream_t st, uint32_t B, const float* input, const float* target) {
	if (dp) training_step_dp(st, B, input, target);
	else if (peer_attached) training_step_peer(st, B, input, target);
	else if (overlapped_ok()) training_step_overlapped(st, B, input, target, true);
	else training_step_sequential(st, B, input, target, true);
}

// tile and layer-wise engines: the pass, the loss sum, then Adam (reference trainer.h:163-190)
void TrainerHost::training_step_sequential(hipStream_t st, uint32_t B, const float* input, const float* target, bool run_optimizer) {
	mark(st, 0);
	model->fwd_bwd(st, ws, B, input, target, n_output_dims, loss_scale, w16.p, nullptr, nullptr, g32.as<float>(),
	               [&](int ph) { mark(st, ph); });
	launch_sum(st, ws.loss_partial.as<float>(), ws.n_loss_partials, d_loss.as<float>());
	mark(st, 4);
	last_B = B;
	if (run_optimizer) optimizer_step(st);
}


// Training step of the fused engine in three launches on one stream (the reference's step is ~10
// kernels plus side streams, trainer.h:163-190): the fused grid+MLP kernel; the grid backward,
// whose 16 extra workgroups (on CUs the grid items leave free) reduce the fused kernel's
// network-gradient slabs and the loss and -- with the optimizer -- run Adam on the network and
// write the next step's weight image; then either Adam over the grid parameters summing the grid
// backward's chunk slabs on the fly, or (run_optimizer = false: the multi-GPU path, whose
// all-reduce sits between the gradients and Adam) the slab reduction into the fp32 gradient.
// Summation orders are the same either way (bit-identical parameters).
void TrainerHost::training_step_overlapped(hipStream_t st, uint32_t B, const float* input, const float* target, bool run_optimizer,
                                           float* grad_out, bool skip_reduce) {
	NetworkHost& m = *model;
	float* const gsum = (grad_out && !run_optimizer) ? grad_out : g32.as<float>();
	mark(st, 0);
	const void* enc_soa = nullptr;
	if (m.sw.split_encode) {  // A/B experiment: the encoding as its own pass, read by the fused kernel
		const GridEncodingHost& g = *m.grid;
		ws.enc16.reserve((size_t)m.mlp.n_input * B * 2);
		launch_grid_fwd(st, g.desc.n_pos_dims, g.desc.n_features_per_level, g.desc.hash_type, B, g.desc.n_levels, input, g.desc.n_pos_dims,
		                (const uint8_t*)w16.p + n_mlp * 2, ws.enc16.p, true, 0, g.dev_levels(), g.hash_grid(), g.desc.interp, g.opts());
		enc_soa = ws.enc16.p;
	}
	m.fused_kernel(st, ws, B, input, target, n_output_dims, loss_scale, w16.p, false, nullptr, nullptr, enc_soa);
	mark(st, 1);
	if (run_optimizer) ++adam_step;
	GridBwdEpilogue ep{};
	ep.enabled = 1;
	ep.apply_adam = run_optimizer ? 1 : 0;
	ep.adam_mlp = run_optimizer ? adam_args_table(st, adam_step) : adam_args();
	ep.adam_mlp.n = (uint32_t)n_mlp;
	ep.buf = AdamBuffers{w32.as<float>(), w16.as<_Float16>(), gsum, g16.as<_Float16>(), m1.as<float>(), m2.as<float>(),
	                     steps.as<uint32_t>()};
	ep.n_mlp_groups = mlp_tail_groups();
	ep.n_mlp = (uint32_t)n_mlp;
	ep.d_loss = d_loss.as<float>();
	TCNN_CHECK(n_mlp % 4 == 0, "network parameter count must be a multiple of 4");
	m.grid_backward(st, ws, B, input, &ep);
	GridEncodingHost& g = *m.grid;
	if (run_optimizer) {
		// binned levels: Adam applied by the accumulate pass; LDS levels: Adam summing their slabs
		GridAccAdam ga{};
		ga.a = adam_args_table(st, adam_step);
		ga.buf = ep.buf;
		ga.param_base = (uint32_t)n_mlp;
		ga.write_grad32 = 0;  // the fp16 gradients (reference m_param_gradients) are written; the fp32 sums are not needed
		g.backward_acc(st, ws.gbw, B, ws.dLdenc.p, 0, 0, g32.as<float>() + n_mlp, &ga);
		mark(st, 2);
		AdamArgs ag = adam_args_table(st, adam_step);
		ag.n = (uint32_t)n_mlp + g.n_lds_params;
		ag.begin = (uint32_t)n_mlp;
		ag.part = ws.gbw.partial.as<float>();
		ag.n_parts = ws.gbw.n_chunks;
		ag.part_stride = g.n_lds_params;
		ag.part_map = g.slab_map(ws.gbw.plan);
		if (!g.plans[0].slices.empty())
			launch_adam(st, ag, w32.as<float>(), w16.p, g32.as<float>(), g16.p, m1.as<float>(), m2.as<float>(), steps.as<uint32_t>());
	} else {
		g.backward_acc(st, ws.gbw, B, ws.dLdenc.p, 0, 0, gsum + n_mlp);
		mark(st, 2);
		if (!skip_reduce) g.reduce_items(st, ws.gbw, gsum + n_mlp);
	}
	mark(st, 3);
	last_B = B;
}

// Captured step graphs, keyed by everything the step's kernels read (graph_key); a few are kept so
// a caller cycling through a handful of batch buffers replays one graph per buffer.
struct TrainerHost::StepGraph {
	static constexpr size_t MAX_GRAPHS = 8;
	hipStream_t cs = nullptr;  // capture / replay stream (the caller's may be the legacy null stream)
	hipEvent_t e0 = nullptr, e1 = nullptr;
	std::vector<std::pair<std::vector<uint64_t>, hipGraphExec_t>> execs;  // most recently used last
	StepGraph() {
		TCNN_HIP_CHECK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
		TCNN_HIP_CHECK(hipEventCreateWithFlags(&e0, hipEventDisableTiming));
		TCNN_HIP_CHECK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
	}
	~StepGraph() {
		for (auto& e : execs) (void)hipGraphExecDestroy(e.second);
		(void)hipEventDestroy(e0);
		(void)hipEventDestroy(e1);
		(void)hipStreamDestroy(cs);
	}
	hipGraphExec_t find(const std::vector<uint64_t>& key) {
		for (size_t i = 0; i < execs.size(); ++i)
			if (execs[i].first == key) {
				auto e = execs[i];
				execs.erase(execs.begin() + i);
				execs.push_back(e);
				return e.second;
			}
		return nullptr;
	}
};

TrainerHost::~TrainerHost() {
	if (graph) (void)hipDeviceSynchronize();  // replays may still run on the graph's stream
}

void TrainerHost::set_graph(bool on) {
	if (!on && graph) {
		TCNN_HIP_CHECK(hipDeviceSynchronize());  // replays run on the callers' streams
		graph.reset();
	}
	use_graph = on;
}

std::vector<uint64_t> TrainerHost::graph_key(uint32_t B, const float* input, const float* target) const {
	std::vector<uint64_t> k = {B, (uint64_t)(uintptr_t)input, (uint64_t)(uintptr_t)target, (uint64_t)ftable_valid,
	                           (uint64_t)(uintptr_t)w32.p, (uint64_t)(uintptr_t)w16.p, (uint64_t)(uintptr_t)g16.p,
	                           (uint64_t)(uintptr_t)g32.p, (uint64_t)(uintptr_t)m1.p, (uint64_t)(uintptr_t)m2.p,
	                           (uint64_t)(uintptr_t)steps.p, (uint64_t)(uintptr_t)d_loss.p, (uint64_t)(uintptr_t)d_ftable.p,
	                           (uint64_t)(uintptr_t)ws.dLdenc.p, (uint64_t)(uintptr_t)ws.wgrad_partial.p,
	                           (uint64_t)(uintptr_t)ws.loss_partial.p, (uint64_t)(uintptr_t)ws.wimage.p,
	                           (uint64_t)(uintptr_t)ws.gbw.partial.p, (uint64_t)(uintptr_t)ws.gbw.recs.p,
	                           (uint64_t)(uintptr_t)ws.gbw.dir.p, (uint64_t)(uintptr_t)ws.gbw.dysum.p, ws.n_fused_blocks,
	                           ws.gbw.n_chunks, (uint64_t)overlapped_ok(), (uint64_t)(uintptr_t)dp, (uint64_t)dp_sharded, dp_per,
	                           (uint64_t)(uintptr_t)ws.enc16.p, (uint64_t)(uintptr_t)ws.acts.p, (uint64_t)(uintptr_t)ws.delta0.p,
	                           (uint64_t)(uintptr_t)ws.delta1.p, (uint64_t)(uintptr_t)ws.dout16.p, (uint64_t)(uintptr_t)ws.out16.p,
	                           (uint64_t)(uintptr_t)ws.red_tmp.p, (uint64_t)(uintptr_t)ws.tile_wT.p, (uint64_t)(uintptr_t)ws.loss_sum.p,
	                           ws.n_loss_partials, (uint64_t)(uintptr_t)peer.get(), (uint64_t)peer_attached};
	// every scalar the step's kernels take from the trainer (AdamArgs holds no pointer here)
	const AdamArgs a = adam_args();
	const size_t n = sizeof(AdamArgs) / 8 + 1;
	std::vector<uint64_t> ab(n, 0);
	std::memcpy(ab.data(), &a, sizeof(AdamArgs));
	k.insert(k.end(), ab.begin(), ab.end());
	const GridOpts o = model->grid ? model->grid->opts() : GridOpts{};  // OneBlob / Identity encodings: no grid
	uint32_t ml = 0;
	std::memcpy(&ml, &o.max_level, 4);
	k.insert(k.end(), {(uint64_t)ml, (uint64_t)(uintptr_t)o.max_level_gpu, o.stochastic, o.n_features, o.active, o.inrange_index});
	uint32_t ls = 0, gs = 0;
	std::memcpy(&ls, &loss_scale, 4);
	std::memcpy(&gs, &grad_scale, 4);
	k.insert(k.end(), {(uint64_t)ls, (uint64_t)gs});
	return k;
}

bool TrainerHost::training_step_graph(hipStream_t st, uint32_t B, const float* input, const float* target) {
	// the single-GPU fused step's first step builds the weight image eagerly (the replays then read it)
	const bool image_step = overlapped_ok() && !dp && !peer_attached;
	if (adam_step + 1 >= GRAPH_STEPS || (image_step && !ws.wimage_valid)) return false;
	if (peer_attached) peer_check();
	if (ftable_valid < GRAPH_STEPS || ftable_b1 != adam.beta1 || ftable_b2 != adam.beta2)
		(void)adam_args_table(st, GRAPH_STEPS, GRAPH_STEPS);
	if (!graph) graph = std::make_unique<StepGraph>();
	std::vector<uint64_t> key = graph_key(B, input, target);
	hipGraphExec_t exec = graph->find(key);
	if (!exec) {
		// eager step first (sizes every workspace for this B, so the capture allocates nothing)
		step_eager(st, B, input, target);
		key = graph_key(B, input, target);
		TCNN_HIP_CHECK(hipStreamSynchronize(st));
		TCNN_HIP_CHECK(hipStreamSynchronize(graph->cs));
		if (graph->execs.size() >= StepGraph::MAX_GRAPHS) {
			(void)hipGraphExecDestroy(graph->execs.front().second);
			graph->execs.erase(graph->execs.begin());
		}
		const uint32_t step0 = adam_step, ftv0 = ftable_valid, lb0 = last_B;
		const bool wv0 = ws.wimage_valid, dps0 = dp_state_partial;
		hipGraph_t g = nullptr;
		const bool tim = timer.enabled;
		timer.enabled = false;  // no phase events inside the graph
		TCNN_HIP_CHECK(hipStreamBeginCapture(graph->cs, hipStreamCaptureModeThreadLocal));
		step_eager(graph->cs, B, input, target);
		TCNN_HIP_CHECK(hipStreamEndCapture(graph->cs, &g));
		timer.enabled = tim;
		adam_step = step0;  // the capture ran nothing
		ftable_valid = ftv0;
		last_B = lb0;
		ws.wimage_valid = wv0;
		dp_state_partial = dps0;
		hipGraphExec_t e = nullptr;
		const hipError_t err = hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
		(void)hipGraphDestroy(g);
		TCNN_HIP_CHECK(err);
		graph->execs.emplace_back(key, e);
		++graph_captures;
		return true;
	}
	// replayed straight on the caller's stream (the legacy null stream included): no private stream,
	// no event joins -- captured on graph->cs only because a capture needs a non-null stream
	TCNN_HIP_CHECK(hipGraphLaunch(exec, st));
	// the host-side effects of the eager step
	++adam_step;
	ws.wimage_valid = image_step;  // the data-parallel steps leave the weight image to be rebuilt by the next step
	if ((dp && dp_sharded) || peer_attached) dp_state_partial = true;
	last_B = B;
	++graph_replays;
	return true;
}

hipEvent_t PhaseTimer::get() {
	if (next == pool.size()) {
		hipEvent_t e;
		TCNN_HIP_CHECK(hipEventCreate(&e));
		pool.push_back(e);
	}
	return pool[next++];
}

PhaseTimer::~PhaseTimer() {
	for (auto e : pool) (void)hipEventDestroy(e);
}

void TrainerHost::mark(hipStream_t st, int phase) {
	if (!timer.enabled || !timer.sampling || timer.marks.empty()) return;
	const int idx = (int)timer.next;
	TCNN_HIP_CHECK(hipEventRecord(timer.get(), st));
	timer.marks.back()[phase] = idx;
}

void TrainerHost::profile_end(double* ms, uint32_t n_phases, uint32_t* n_steps) {
	TCNN_HIP_CHECK(hipDeviceSynchronize());
	const uint32_t P = std::min<uint32_t>(n_phases, PhaseTimer::N_PHASES);
	for (uint32_t p = 0; p < n_phases; ++p) ms[p] = 0.0;
	std::vector<uint32_t> cnt(P, 0);
	for (auto& m : timer.marks) {
		for (uint32_t p = 0; p < P; ++p) {
			if (m[p] < 0 || m[p + 1] < 0) continue;
			float t = 0.0f;
			TCNN_HIP_CHECK(hipEventElapsedTime(&t, timer.pool[m[p]], timer.pool[m[p + 1]]));
			ms[p] += t;
			++cnt[p];
		}
	}
	for (uint32_t p = 0; p < P; ++p)
		if (cnt[p]) ms[p] /= cnt[p];
	if (n_steps) *n_steps = P ? cnt[0] : 0;
	timer.enabled = false;
	timer.reset();
}

AdamArgs TrainerHost::adam_args() const {
	AdamArgs a{};
	a.n = (uint32_t)n_params;
	a.n_matrix = (uint32_t)n_mlp;  // layer_sizes() of the network only (grid.h:1084-1088)
	a.loss_scale = loss_scale;
	a.grad_scale = grad_scale;
	a.lr = adam.learning_rate;
	a.beta1 = adam.beta1;
	a.beta2 = adam.beta2;
	a.eps = adam.epsilon;
	a.l2_reg = adam.l2_reg;
	a.rel_decay = adam.relative_decay;
	a.abs_decay = adam.absolute_decay;
	a.clip = adam.clipping_magnitude;
	a.nonmat_lr_factor = adam.non_matrix_learning_rate_factor;
	a.lower_lr_bound = 0.0f;
	a.upper_lr_bound = std::numeric_limits<float>::max();
	if (adam.adabound) {
		a.lower_lr_bound = 0.1f - 0.1f / ((1 - adam.beta2) * (float)adam_step + 1);
		a.upper_lr_bound = 0.1f + 0.1f / ((1 - adam.beta2) * (float)adam_step);
	}
	a.opt_matrix = adam.optimize_matrix_params;
	a.opt_nonmatrix = adam.optimize_non_matrix_params;
	int e = 0;
	a.inv_loss_scale = (std::frexp(loss_scale, &e) == 0.5f) ? 1.0f / loss_scale : 0.0f;  // exact for powers of two
	return a;
}

// Data-parallel step in two parts, so the caller can all-reduce the network gradients while the
// grid backward runs (part 0: fused grid+MLP kernel, network-gradient column sums into
// g32[0, n_mlp) and the loss sum; part 1: grid backward + slab reduction into g32[n_mlp, n)). Same
// kernels and summation orders as training_step(run_optimizer = false). The layer-wise engine does
// its whole pass in part 0.
void TrainerHost::training_step_part(hipStream_t st, uint32_t B, const float* input, const float* target, int part) {
	TCNN_CHECK(B % BATCH_GRANULARITY == 0, "training_step: batch size must be a multiple of 256");
	TCNN_CHECK(part == 0 || part == 1, "training_step_part: part must be 0 or 1");
	NetworkHost& m = *model;
	if (!overlapped_ok()) {
		if (part == 0) training_step(st, B, input, target, false);
		return;
	}
	if (part == 0) {
		m.fused_kernel(st, ws, B, input, target, n_output_dims, loss_scale, w16.p, false);
		launch_column_sums(st, ws.wgrad_partial.as<float>(), ws.n_fused_blocks, (uint32_t)n_mlp, g32.as<float>());
		launch_sum(st, ws.loss_partial.as<float>(), ws.n_loss_partials, d_loss.as<float>());
		last_B = B;
		return;
	}
	TCNN_CHECK(last_B == B, "training_step_part: part 1 must follow part 0 of the same batch");
	m.grid_backward(st, ws, B, input);
	m.grid->backward_acc(st, ws.gbw, B, ws.dLdenc.p, 0, 0, g32.as<float>() + n_mlp);
	m.grid->reduce_items(st, ws.gbw, g32.as<float>() + n_mlp);
}

AdamArgs TrainerHost::adam_args_table(hipStream_t st, uint32_t upto, uint32_t reserve) {
	AdamArgs a = adam_args();
	if (ftable_b1 != adam.beta1 || ftable_b2 != adam.beta2) {  // hyper-parameters changed: recompute all
		ftable_valid = 0;
		ftable_b1 = adam.beta1;
		ftable_b2 = adam.beta2;
	}
	if (std::max(upto, reserve) > ftable_cap) {
		ftable_cap = std::max((std::max(upto, reserve) + 1023u) / 1024u * 1024u, std::max(1024u, 2 * ftable_cap));
		TCNN_HIP_CHECK(hipStreamSynchronize(st));  // the old table may still be read by queued work
		d_ftable.reserve((size_t)ftable_cap * 4);
		ftable_valid = 0;
	}
	if (std::max(upto, reserve) > ftable_valid) {
		// the factors depend only on t and the betas, sqrt(1 - b2^t) / (1 - b1^t) (adam.h:110-113),
		// computed 1024 steps ahead on the host with the C library's powf / sqrtf -- one libm for
		// every step, the same one the CPU restatement uses, so the Adam update is bit-exact against it
		// (a device powf differs from glibc's in the last bit for some t)
		const uint32_t ahead = std::min(ftable_cap, (std::max(upto, reserve) + 1023u) / 1024u * 1024u);
		h_ftable.resize(ahead);
		for (uint32_t t = ftable_valid + 1; t <= ahead; ++t)
			h_ftable[t - 1] = std::sqrt(1.0f - std::pow(adam.beta2, (float)t)) / (1.0f - std::pow(adam.beta1, (float)t));
		TCNN_HIP_CHECK(hipMemcpyAsync(d_ftable.as<float>() + ftable_valid, h_ftable.data() + ftable_valid, (size_t)(ahead - ftable_valid) * 4,
		                              hipMemcpyHostToDevice, st));
		TCNN_HIP_CHECK(hipStreamSynchronize(st));  // h_ftable may grow (reallocate) before the next fill
		ftable_valid = ahead;
	}
	a.factor_table = d_ftable.as<float>();
	a.factor_n = ftable_valid;
	return a;
}

void TrainerHost::optimizer_step(hipStream_t st) {  // AdamOptimizer::step, adam.h:150-188
	++adam_step;
	const AdamArgs a = adam_args_table(st, adam_step);
	launch_adam(st, a, w32.as<float>(), w16.p, g32.as<float>(), g16.p, m1.as<float>(), m2.as<float>(), steps.as<uint32_t>());
	ws.wimage_valid = false;
}

std::unique_ptr<TrainerFwdCtx> TrainerHost::forward(hipStream_t st, uint32_t B, const float* input, const float* target, const float* pdf,
                                                    const void* ext_dLdy16, bool prep_dinput, const float* perturbation) {
	TCNN_CHECK(B % BATCH_GRANULARITY == 0, "forward: batch size must be a multiple of 256");
	TCNN_CHECK(ext_dLdy16 || target, "forward: a target (or an external dL/dy) is required");
	NetworkHost& m = *model;
	const uint32_t OUTP = m.mlp.padded_output;
	auto c = std::make_unique<TrainerFwdCtx>();
	c->B = B;
	c->out16.reserve((size_t)B * OUTP * 2);
	c->layout = m.forward_keep(st, ws, B, input, w16.p, c->out16.p, prep_dinput, c->keep);
	if (ext_dLdy16) {  // trainer.h:126-130: the caller's dL/dy replaces the loss
		c->ext = ext_dLdy16;
	} else {
		c->dLdy16.reserve((size_t)B * OUTP * 2);
		c->n_lpart = relative_l2_n_blocks(B, OUTP);
		c->lpart.reserve((size_t)c->n_lpart * 4);
		const void* loss_in = c->out16.p;
		if (perturbation) {  // trainer.h:114-123: the loss (and its dL/dy) on the perturbed output
			c->pert16.reserve((size_t)B * OUTP * 2);
			launch_add_perturbation(st, B * OUTP, c->out16.p, perturbation, c->pert16.p);
			loss_in = c->pert16.p;
		}
		launch_relative_l2_partial(st, B, OUTP, n_output_dims, loss_scale, loss_in, target, c->dLdy16.p, c->lpart.as<float>(),
		                           m.loss_l2, pdf);
	}
	ws.wimage_valid = false;  // forward_keep may have packed the image in place
	return c;
}

void TrainerHost::backward(hipStream_t st, const TrainerFwdCtx& c, uint32_t B, const float* input, float* dL_dinput, int gradient_mode) {
	TCNN_CHECK(B == c.B, "backward: batch size differs from the forward's");
	// Accumulate: this backward's gradients into a scratch sum, added afterwards (trainer.h:146-153).
	// Ignore: the same scratch, never added -- the parameter gradients stay as they were and only
	// dL/dinput is delivered (the engine's fused backward computes both in one pass).
	float* dst = g32.as<float>();
	if (gradient_mode != 0) {
		g32_acc.reserve(n_params * 4);
		dst = g32_acc.as<float>();
	}
	model->fwd_bwd(st, ws, B, input, nullptr, n_output_dims, 1.0f, w16.p, c.dLdy(), nullptr, dst, nullptr, dL_dinput,
	               c.keep.p ? c.keep.p : nullptr, c.layout);
	if (gradient_mode == 1) launch_add_f32(st, dst, g32.as<float>(), n_params);
	ws.wimage_valid = false;
	last_B = B;
}

float TrainerHost::ctx_loss(hipStream_t st, const TrainerFwdCtx& c) {  // trainer.h:205-211
	if (c.ext) return 0.0f;  // no loss was evaluated (the reference's L stays unwritten)
	launch_sum(st, c.lpart.as<float>(), c.n_lpart, d_loss.as<float>());
	return loss(st);
}

void TrainerHost::optimizer_step_range(hipStream_t st, uint64_t begin, uint64_t end) {
	TCNN_CHECK(begin <= end && end <= n_params, "optimizer_step_range: range outside the parameter vector");
	++adam_step;
	AdamArgs a = adam_args_table(st, adam_step);
	a.begin = (uint32_t)begin;
	a.n = (uint32_t)end;
	launch_adam(st, a, w32.as<float>(), w16.p, g32.as<float>(), g16.p, m1.as<float>(), m2.as<float>(), steps.as<uint32_t>());
	ws.wimage_valid = false;
}

float TrainerHost::loss(hipStream_t st) {
	float v = 0.0f;
	TCNN_HIP_CHECK(hipMemcpyAsync(&v, d_loss.p, 4, hipMemcpyDeviceToHost, st));
	TCNN_HIP_CHECK(hipStreamSynchronize(st));
	return v;
}

void TrainerHost::inference(hipStream_t st, uint32_t B, const float* input, float* out) {
	const uint32_t OUTP = model->mlp.padded_output;
	ws.out16.reserve((size_t)B * OUTP * 2);
	model->inference(st, ws, B, input, w16.p, ws.out16.p, /*trust_image=*/true);
	launch_trim_cast(st, B, OUTP, n_output_dims, ws.out16.p, out);
}

}  // namespace tcnn_amd
