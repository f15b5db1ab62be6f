// tiny-cuda-nn/multi_stream.h -- SyncedMultiStream (reference include/tiny-cuda-nn/multi_stream.h:
// StreamAndEvent :41-94, MultiStream :96-148, the per-parent pools :150-194, SyncedMultiStream
// :196-259) on HIP streams and events, header-only: a fork of `n_streams - 1` auxiliary streams that
// wait for the parent's work so far, and a join on destruction (the parent waits for every
// auxiliary stream). Auxiliary stream sets are pooled per parent stream and reused.
#pragma once

#include <memory>
#include <mutex>
#include <stack>
#include <unordered_map>
#include <vector>

#include "common.h"
#include "gpu_memory.h"

namespace tcnn {

struct StreamAndEvent {  // multi_stream.h:41-94
	StreamAndEvent() {
		HIP_CHECK_THROW(hipStreamCreate(&m_stream));
		HIP_CHECK_THROW(hipEventCreateWithFlags(&m_event, hipEventDisableTiming));
	}
	~StreamAndEvent() {
		if (m_stream) {
			tcnn_free_workspace_arena(m_stream);
			(void)hipStreamDestroy(m_stream);
		}
		if (m_event) (void)hipEventDestroy(m_event);
	}
	StreamAndEvent(const StreamAndEvent&) = delete;
	StreamAndEvent& operator=(const StreamAndEvent&) = delete;
	hipStream_t get() const { return m_stream; }
	void wait_for(hipEvent_t e) { HIP_CHECK_THROW(hipStreamWaitEvent(m_stream, e, 0)); }
	void wait_for(hipStream_t s) {
		HIP_CHECK_THROW(hipEventRecord(m_event, s));
		wait_for(m_event);
	}
	void signal(hipStream_t s) {
		HIP_CHECK_THROW(hipEventRecord(m_event, m_stream));
		HIP_CHECK_THROW(hipStreamWaitEvent(s, m_event, 0));
	}

private:
	hipStream_t m_stream = nullptr;
	hipEvent_t m_event = nullptr;
};

struct MultiStream {  // multi_stream.h:96-148
	explicit MultiStream(size_t n) : m_streams(n) { HIP_CHECK_THROW(hipEventCreateWithFlags(&m_event, hipEventDisableTiming)); }
	~MultiStream() { (void)hipEventDestroy(m_event); }
	MultiStream(const MultiStream&) = delete;
	MultiStream& operator=(const MultiStream&) = delete;
	void wait_for(hipStream_t s) {
		HIP_CHECK_THROW(hipEventRecord(m_event, s));
		for (auto& st : m_streams) st.wait_for(m_event);
	}
	void signal(hipStream_t s) {
		for (auto& st : m_streams) st.signal(s);
	}
	hipStream_t get(size_t i) const { return m_streams.at(i).get(); }
	size_t size() const { return m_streams.size(); }

private:
	std::vector<StreamAndEvent> m_streams;
	hipEvent_t m_event = nullptr;
};

namespace detail {
struct MultiStreamPool {
	std::mutex mu;
	std::unordered_map<hipStream_t, std::stack<std::shared_ptr<MultiStream>>> by_parent;
};
inline MultiStreamPool& multi_stream_pool() {
	static auto* p = new MultiStreamPool{};
	return *p;
}
}  // namespace detail

// multi_stream.h:174-194
inline std::shared_ptr<MultiStream> reserve_multi_stream(hipStream_t parent, size_t n_streams) {
	auto& P = detail::multi_stream_pool();
	std::lock_guard<std::mutex> lk(P.mu);
	auto& stack = P.by_parent[parent];
	if (stack.empty() || stack.top()->size() < n_streams) return std::make_shared<MultiStream>(n_streams);
	auto r = stack.top();
	stack.pop();
	return r;
}
inline void return_multi_stream(hipStream_t parent, std::shared_ptr<MultiStream> ms) {
	auto& P = detail::multi_stream_pool();
	std::lock_guard<std::mutex> lk(P.mu);
	P.by_parent[parent].push(std::move(ms));
}
inline void free_multi_streams(hipStream_t parent) {  // multi_stream.h:164-172
	std::stack<std::shared_ptr<MultiStream>> drop;
	{
		auto& P = detail::multi_stream_pool();
		std::lock_guard<std::mutex> lk(P.mu);
		auto it = P.by_parent.find(parent);
		if (it == P.by_parent.end()) return;
		drop = std::move(it->second);
		P.by_parent.erase(it);
	}
}

struct SyncedMultiStream {  // multi_stream.h:196-259
	SyncedMultiStream() = default;
	SyncedMultiStream(hipStream_t stream, size_t n_streams) : m_main_stream{stream}, m_n_streams{n_streams} {
		if (m_n_streams == 0) throw std::runtime_error{"SyncedMultiStream: must request at least one stream"};
		if (m_n_streams == 1) return;
		m_multi_stream = reserve_multi_stream(m_main_stream, m_n_streams - 1);
		m_multi_stream->wait_for(m_main_stream);
	}
	~SyncedMultiStream() {
		if (m_multi_stream) {
			m_multi_stream->signal(m_main_stream);
			return_multi_stream(m_main_stream, m_multi_stream);
		}
	}
	SyncedMultiStream(const SyncedMultiStream&) = delete;
	SyncedMultiStream& operator=(const SyncedMultiStream&) = delete;
	SyncedMultiStream(SyncedMultiStream&& other) { *this = std::move(other); }
	SyncedMultiStream& operator=(SyncedMultiStream&& other) {
		std::swap(m_multi_stream, other.m_multi_stream);
		std::swap(m_main_stream, other.m_main_stream);
		std::swap(m_n_streams, other.m_n_streams);
		return *this;
	}
	hipStream_t get(size_t idx) {
		if (m_n_streams == 0) throw std::runtime_error{"SyncedMultiStream: must have at least one stream"};
		if (idx == 0) return m_main_stream;
		if (!m_multi_stream || idx - 1 >= m_multi_stream->size())
			throw std::runtime_error{"SyncedMultiStream: invalid stream index"};
		return m_multi_stream->get(idx - 1);
	}

private:
	std::shared_ptr<MultiStream> m_multi_stream = nullptr;
	hipStream_t m_main_stream = nullptr;
	size_t m_n_streams = 0;
};

}  // namespace tcnn
