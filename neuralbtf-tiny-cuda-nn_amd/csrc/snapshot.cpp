// snapshot.cpp -- Trainer (de)serialisation in the reference's snapshot format.
//
// The reference writes `json::to_msgpack(trainer->serialize(optimizer))` (trainer.h:275-315,
// adam.h:278-299, gpu_memory_json.h:36-71): a msgpack map, keys in std::map (lexicographic) order,
//   n_params          uint
//   optimizer         (optional) map: base_learning_rate float, current_step uint,
//                     first_moments_binary / second_moments_binary bin (fp32 [n]),
//                     param_steps_binary bin (uint32 [n])
//   params_binary     bin: the fp16 inference parameters (PARAMS_T = __half)
//   params_type       "__half"
// nlohmann::json in this image (3.1.1) predates binary values, so the msgpack writer/reader for this
// schema is written out here (big-endian numbers; unsigned ints in their smallest form; floats as
// float32 when exactly representable, as nlohmann 3.9+ does; bin8/16/32 for binaries).
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "runtime.h"

namespace tcnn_amd {
namespace {

struct MsgWriter {
	std::vector<uint8_t> b;
	void u8(uint8_t v) { b.push_back(v); }
	void be(uint64_t v, int n) {
		for (int i = n - 1; i >= 0; --i) b.push_back((uint8_t)(v >> (8 * i)));
	}
	void map(uint32_t n) {
		if (n <= 15) u8((uint8_t)(0x80 | n));
		else if (n <= 0xffff) { u8(0xde); be(n, 2); }
		else { u8(0xdf); be(n, 4); }
	}
	void str(const std::string& s) {
		const size_t n = s.size();
		if (n <= 31) u8((uint8_t)(0xa0 | n));
		else if (n <= 0xff) { u8(0xd9); be(n, 1); }
		else if (n <= 0xffff) { u8(0xda); be(n, 2); }
		else { u8(0xdb); be(n, 4); }
		b.insert(b.end(), s.begin(), s.end());
	}
	void uint(uint64_t v) {
		if (v <= 0x7f) u8((uint8_t)v);
		else if (v <= 0xff) { u8(0xcc); be(v, 1); }
		else if (v <= 0xffff) { u8(0xcd); be(v, 2); }
		else if (v <= 0xffffffffull) { u8(0xce); be(v, 4); }
		else { u8(0xcf); be(v, 8); }
	}
	void flt(double v) {
		const float f = (float)v;
		if ((double)f == v || std::isnan(v)) {
			uint32_t u;
			std::memcpy(&u, &f, 4);
			u8(0xca);
			be(u, 4);
		} else {
			uint64_t u;
			std::memcpy(&u, &v, 8);
			u8(0xcb);
			be(u, 8);
		}
	}
	void bin(const void* p, size_t n) {
		if (n <= 0xff) { u8(0xc4); be(n, 1); }
		else if (n <= 0xffff) { u8(0xc5); be(n, 2); }
		else { u8(0xc6); be(n, 4); }
		const uint8_t* c = (const uint8_t*)p;
		b.insert(b.end(), c, c + n);
	}
};

// Minimal msgpack value tree for the snapshot schema (maps, arrays, strings, numbers, binaries).
struct MsgValue {
	enum Kind { Nil, Bool, UInt, Int, Float, Str, Bin, Map, Arr } kind = Nil;
	uint64_t u = 0;
	int64_t i = 0;
	double f = 0;
	std::string s;  // Str / Bin payload
	std::map<std::string, MsgValue> m;
	std::vector<MsgValue> a;
	double number() const {
		switch (kind) {
			case UInt: return (double)u;
			case Int: return (double)i;
			case Float: return f;
			default: throw std::runtime_error("snapshot: expected a number");
		}
	}
	bool has(const std::string& k) const { return kind == Map && m.count(k); }
	const MsgValue& at(const std::string& k) const {
		TCNN_CHECK(has(k), "snapshot: missing key '" + k + "'");
		return m.find(k)->second;
	}
};

struct MsgReader {
	const uint8_t* p;
	const uint8_t* end;
	uint64_t be(int n) {
		TCNN_CHECK(end - p >= n, "snapshot: truncated msgpack data");
		uint64_t v = 0;
		for (int k = 0; k < n; ++k) v = (v << 8) | *p++;
		return v;
	}
	std::string bytes(uint64_t n) {
		TCNN_CHECK((uint64_t)(end - p) >= n, "snapshot: truncated msgpack data");
		std::string r((const char*)p, (size_t)n);
		p += n;
		return r;
	}
	MsgValue value(int depth = 0) {
		TCNN_CHECK(depth < 16 && p < end, "snapshot: malformed msgpack data");
		const uint8_t t = *p++;
		MsgValue v;
		auto read_map = [&](uint64_t n) {
			v.kind = MsgValue::Map;
			for (uint64_t k = 0; k < n; ++k) {
				MsgValue key = value(depth + 1);
				TCNN_CHECK(key.kind == MsgValue::Str, "snapshot: map keys must be strings");
				v.m[key.s] = value(depth + 1);
			}
		};
		auto read_arr = [&](uint64_t n) {
			v.kind = MsgValue::Arr;
			for (uint64_t k = 0; k < n; ++k) v.a.push_back(value(depth + 1));
		};
		auto read_ext = [&](uint64_t n) {  // ext: type byte, then the payload (kept as binary)
			be(1);
			v.kind = MsgValue::Bin;
			v.s = bytes(n);
		};
		if (t <= 0x7f) { v.kind = MsgValue::UInt; v.u = t; }
		else if ((t & 0xf0) == 0x80) read_map(t & 0x0f);
		else if ((t & 0xf0) == 0x90) read_arr(t & 0x0f);
		else if ((t & 0xe0) == 0xa0) { v.kind = MsgValue::Str; v.s = bytes(t & 0x1f); }
		else if (t >= 0xe0) { v.kind = MsgValue::Int; v.i = (int8_t)t; }
		else switch (t) {
			case 0xc0: break;
			case 0xc2: v.kind = MsgValue::Bool; v.u = 0; break;
			case 0xc3: v.kind = MsgValue::Bool; v.u = 1; break;
			case 0xc4: v.kind = MsgValue::Bin; v.s = bytes(be(1)); break;
			case 0xc5: v.kind = MsgValue::Bin; v.s = bytes(be(2)); break;
			case 0xc6: v.kind = MsgValue::Bin; v.s = bytes(be(4)); break;
			case 0xc7: read_ext(be(1)); break;
			case 0xc8: read_ext(be(2)); break;
			case 0xc9: read_ext(be(4)); break;
			case 0xca: { const uint32_t u = (uint32_t)be(4); float f; std::memcpy(&f, &u, 4); v.kind = MsgValue::Float; v.f = f; break; }
			case 0xcb: { const uint64_t u = be(8); double d; std::memcpy(&d, &u, 8); v.kind = MsgValue::Float; v.f = d; break; }
			case 0xcc: v.kind = MsgValue::UInt; v.u = be(1); break;
			case 0xcd: v.kind = MsgValue::UInt; v.u = be(2); break;
			case 0xce: v.kind = MsgValue::UInt; v.u = be(4); break;
			case 0xcf: v.kind = MsgValue::UInt; v.u = be(8); break;
			case 0xd0: v.kind = MsgValue::Int; v.i = (int8_t)be(1); break;
			case 0xd1: v.kind = MsgValue::Int; v.i = (int16_t)be(2); break;
			case 0xd2: v.kind = MsgValue::Int; v.i = (int32_t)be(4); break;
			case 0xd3: v.kind = MsgValue::Int; v.i = (int64_t)be(8); break;
			case 0xd9: v.kind = MsgValue::Str; v.s = bytes(be(1)); break;
			case 0xda: v.kind = MsgValue::Str; v.s = bytes(be(2)); break;
			case 0xdb: v.kind = MsgValue::Str; v.s = bytes(be(4)); break;
			case 0xdc: read_arr(be(2)); break;
			case 0xdd: read_arr(be(4)); break;
			case 0xde: read_map(be(2)); break;
			case 0xdf: read_map(be(4)); break;
			default: throw std::runtime_error("snapshot: unsupported msgpack type");
		}
		return v;
	}
};

std::vector<uint8_t> d2h(const DevBuf& b, size_t bytes) {
	std::vector<uint8_t> h(bytes);
	if (bytes) TCNN_HIP_CHECK(hipMemcpy(h.data(), b.p, bytes, hipMemcpyDeviceToHost));
	return h;
}

// from_json(json, GPUMemory<T>&) (gpu_memory_json.h:52-71): a binary, or its JSON image
// {"bytes": [u8, ...], "subtype": ...} (nlohmann's binary-as-JSON form)
std::string bin_of(const MsgValue& v, size_t bytes, const char* what) {
	std::string out;
	if (v.kind == MsgValue::Bin) {
		out = v.s;
	} else if (v.kind == MsgValue::Map && v.has("bytes") && v.at("bytes").kind == MsgValue::Arr) {
		const auto& arr = v.at("bytes").a;
		out.resize(arr.size());
		for (size_t i = 0; i < arr.size(); ++i) out[i] = (char)(uint8_t)arr[i].number();
	} else {
		throw std::runtime_error(std::string("snapshot: '") + what + "': Invalid json type: must be either binary or object");
	}
	TCNN_CHECK(out.size() == bytes, std::string("snapshot: '") + what + "' has the wrong size");
	return out;
}

// JSON text snapshot (json::dump of Trainer::serialize, binaries in their {"bytes": [...]} form)
MsgValue from_json_text(const json& j) {
	MsgValue v;
	if (j.is_object()) {
		v.kind = MsgValue::Map;
		for (auto it = j.begin(); it != j.end(); ++it) v.m[it.key()] = from_json_text(it.value());
	} else if (j.is_array()) {
		v.kind = MsgValue::Arr;
		for (const auto& e : j) v.a.push_back(from_json_text(e));
	} else if (j.is_string()) {
		v.kind = MsgValue::Str;
		v.s = j.get<std::string>();
	} else if (j.is_boolean()) {
		v.kind = MsgValue::Bool;
		v.u = j.get<bool>() ? 1 : 0;
	} else if (j.is_number_unsigned()) {
		v.kind = MsgValue::UInt;
		v.u = j.get<uint64_t>();
	} else if (j.is_number_integer()) {
		v.kind = MsgValue::Int;
		v.i = j.get<int64_t>();
	} else if (j.is_number_float()) {
		v.kind = MsgValue::Float;
		v.f = j.get<double>();
	}
	return v;
}

// MsgValue -> nlohmann json, binaries in nlohmann's binary-as-JSON form {"bytes": [...], "subtype": null}
// (json::dump of a binary value in nlohmann >= 3.8; the reference's Trainer::serialize returns json
// holding binaries, trainer.h:275-290) -- the form deserialize() accepts back
json to_json(const MsgValue& v) {
	switch (v.kind) {
		case MsgValue::Nil: return json();
		case MsgValue::Bool: return json(v.u != 0);
		case MsgValue::UInt: return json(v.u);
		case MsgValue::Int: return json(v.i);
		case MsgValue::Float: return json(v.f);
		case MsgValue::Str: return json(v.s);
		case MsgValue::Bin: {
			json bytes = json::array();
			for (unsigned char c : v.s) bytes.push_back((unsigned)c);
			json b = json::object();
			b["bytes"] = std::move(bytes);
			b["subtype"] = json();
			return b;
		}
		case MsgValue::Map: {
			json o = json::object();
			for (const auto& kv : v.m) o[kv.first] = to_json(kv.second);
			return o;
		}
		case MsgValue::Arr: {
			json a = json::array();
			for (const auto& e : v.a) a.push_back(to_json(e));
			return a;
		}
	}
	return json();
}

}  // namespace

std::string TrainerHost::serialize_json(bool with_optimizer) {
	const std::vector<uint8_t> b = serialize(with_optimizer);
	MsgReader r{b.data(), b.data() + b.size()};
	return to_json(r.value()).dump();
}

std::vector<uint8_t> TrainerHost::serialize(bool with_optimizer) {
	TCNN_CHECK(!(with_optimizer && dp_sharded && dp_state_partial),
	           "serialize(optimizer): the sharded data-parallel optimizer state is current only on each rank's shard; "
	           "gather it first (tcnn_trainer_dp_gather_state)");
	TCNN_HIP_CHECK(hipDeviceSynchronize());
	const size_t n = n_params;
	MsgWriter w;
	w.map(with_optimizer ? 4 : 3);
	w.str("n_params");
	w.uint(n);
	if (with_optimizer) {  // AdamOptimizer::serialize (adam.h:278-286)
		w.str("optimizer");
		w.map(5);
		w.str("base_learning_rate");
		w.flt(adam.learning_rate);
		w.str("current_step");
		w.uint(adam_step);
		const auto m1h = d2h(m1, n * 4), m2h = d2h(m2, n * 4), sth = d2h(steps, n * 4);
		w.str("first_moments_binary");
		w.bin(m1h.data(), m1h.size());
		w.str("param_steps_binary");
		w.bin(sth.data(), sth.size());
		w.str("second_moments_binary");
		w.bin(m2h.data(), m2h.size());
	}
	const auto ph = d2h(w16, n * 2);
	w.str("params_binary");
	w.bin(ph.data(), ph.size());
	w.str("params_type");
	w.str("__half");
	return std::move(w.b);
}

void TrainerHost::deserialize(const void* data, size_t size) {
	// training steps may still be queued on the caller's (possibly non-blocking) stream
	TCNN_HIP_CHECK(hipDeviceSynchronize());
	MsgValue root;
	if (size > 0 && ((const char*)data)[0] == '{') {  // JSON text
		root = from_json_text(json::parse(std::string((const char*)data, size)));
	} else {
		MsgReader r{(const uint8_t*)data, (const uint8_t*)data + size};
		root = r.value();
	}
	TCNN_CHECK(root.kind == MsgValue::Map, "snapshot: top level must be a map");
	const size_t n = n_params;
	const std::string type = root.has("params_type") ? root.at("params_type").s : "__half";
	const MsgValue& pb = root.at("params_binary");
	if (type == "float") {  // trainer.h:292-294: fp32 params -> full precision + fp16 copy
		const std::string b = bin_of(pb, n * 4, "params_binary");
		std::vector<float> host(n);
		std::memcpy(host.data(), b.data(), n * 4);
		set_params_full_precision(host.data(), n);
	} else if (type == "__half") {  // trainer.h:295-304: fp16 params; full precision = (float)half
		const std::string b = bin_of(pb, n * 2, "params_binary");
		TCNN_HIP_CHECK(hipMemcpy(w16.p, b.data(), n * 2, hipMemcpyHostToDevice));
		launch_cast_f16_f32(nullptr, w16.p, w32.as<float>(), n);
		TCNN_HIP_CHECK(hipDeviceSynchronize());
		ws.wimage_valid = false;
	} else {
		throw std::runtime_error("Trainer: snapshot parameters must be of type float of __half");
	}
	if (root.has("optimizer")) {  // AdamOptimizer::deserialize (adam.h:288-299)
		const MsgValue& o = root.at("optimizer");
		TCNN_HIP_CHECK(hipMemcpy(m1.p, bin_of(o.at("first_moments_binary"), n * 4, "first_moments_binary").data(), n * 4,
		                         hipMemcpyHostToDevice));
		TCNN_HIP_CHECK(hipMemcpy(m2.p, bin_of(o.at("second_moments_binary"), n * 4, "second_moments_binary").data(), n * 4,
		                         hipMemcpyHostToDevice));
		if (o.has("param_steps_binary"))
			TCNN_HIP_CHECK(hipMemcpy(steps.p, bin_of(o.at("param_steps_binary"), n * 4, "param_steps_binary").data(), n * 4,
			                         hipMemcpyHostToDevice));
		else
			TCNN_HIP_CHECK(hipMemset(steps.p, 0, n * 4));
		adam_step = (uint32_t)o.at("current_step").number();
		adam.learning_rate = (float)o.at("base_learning_rate").number();
	}
	TCNN_HIP_CHECK(hipDeviceSynchronize());
}

}  // namespace tcnn_amd
