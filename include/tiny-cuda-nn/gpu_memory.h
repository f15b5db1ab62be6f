// tiny-cuda-nn/gpu_memory.h -- GPUMemory<T> (reference include/tiny-cuda-nn/gpu_memory.h:60-390):
// an owning, move-only device array; and the stream-ordered workspace arena (gpu_memory.h:426-754:
// GPUMemoryArena::Allocation, allocate_workspace, allocate_workspace_and_distribute,
// free_gpu_memory_arena) over the engine's arenas (tcnn_workspace_*, csrc/arena.cpp: one virtual
// address range per stream with physical memory mapped at its end as it grows, so workspace
// addresses survive growth).
#pragma once

#include <cstring>
#include <tuple>
#include <utility>
#include <vector>

#include "common.h"

namespace tcnn {

template <typename T>
class GPUMemory {
public:
	GPUMemory() {}
	explicit GPUMemory(size_t size, bool managed = false) : m_managed{managed} { resize(size); }
	GPUMemory(GPUMemory<T>&& other) { *this = std::move(other); }
	GPUMemory<T>& operator=(GPUMemory<T>&& other) {
		std::swap(m_data, other.m_data);
		std::swap(m_size, other.m_size);
		std::swap(m_managed, other.m_managed);
		return *this;
	}
	GPUMemory(const GPUMemory<T>&) = delete;
	GPUMemory<T>& operator=(const GPUMemory<T>&) = delete;
	~GPUMemory() { free_memory(); }

	void free_memory() {
		if (m_data) (void)hipFree(m_data);
		m_data = nullptr;
		m_size = 0;
	}

	// gpu_memory.h:168-189: contents are not preserved
	void resize(const size_t size) {
		if (m_size == size) return;
		free_memory();
		if (size == 0) return;
		if (m_managed) HIP_CHECK_THROW(hipMallocManaged((void**)&m_data, size * sizeof(T)));
		else HIP_CHECK_THROW(hipMalloc((void**)&m_data, size * sizeof(T)));
		m_size = size;
	}
	void enlarge(const size_t size) {
		if (size > m_size) resize(size);
	}

	void memset(const int value, const size_t num_elements, const size_t offset = 0) {
		CHECK_THROW(num_elements + offset <= m_size);
		HIP_CHECK_THROW(hipMemset(m_data + offset, value, num_elements * sizeof(T)));
	}
	void memset(const int value) { memset(value, m_size); }

	void copy_from_host(const T* host_data, const size_t num_elements) {
		CHECK_THROW(num_elements <= m_size);
		HIP_CHECK_THROW(hipMemcpy(m_data, host_data, num_elements * sizeof(T), hipMemcpyHostToDevice));
	}
	void copy_from_host(const std::vector<T>& data, const size_t num_elements) {
		CHECK_THROW(data.size() >= num_elements);
		copy_from_host(data.data(), num_elements);
	}
	void copy_from_host(const T* data) { copy_from_host(data, m_size); }
	void copy_from_host(const std::vector<T>& data) { copy_from_host(data.data(), std::min(m_size, data.size())); }
	void enlarge_and_copy_from_host(const T* data, const size_t num_elements) {
		enlarge(num_elements);
		copy_from_host(data, num_elements);
	}
	void enlarge_and_copy_from_host(const std::vector<T>& data) { enlarge_and_copy_from_host(data.data(), data.size()); }
	void resize_and_copy_from_host(const T* data, const size_t num_elements) {
		resize(num_elements);
		copy_from_host(data, num_elements);
	}
	void resize_and_copy_from_host(const std::vector<T>& data) { resize_and_copy_from_host(data.data(), data.size()); }

	void copy_to_host(T* host_data, const size_t num_elements) const {
		CHECK_THROW(num_elements <= m_size);
		HIP_CHECK_THROW(hipMemcpy(host_data, m_data, num_elements * sizeof(T), hipMemcpyDeviceToHost));
	}
	void copy_to_host(std::vector<T>& data, const size_t num_elements) const {
		CHECK_THROW(data.size() >= num_elements);
		copy_to_host(data.data(), num_elements);
	}
	void copy_to_host(T* data) const { copy_to_host(data, m_size); }
	void copy_to_host(std::vector<T>& data) const { copy_to_host(data.data(), std::min(m_size, data.size())); }

	void copy_from_device(const GPUMemory<T>& other, const size_t size) {
		CHECK_THROW(size <= other.m_size);
		enlarge(size);
		HIP_CHECK_THROW(hipMemcpy(m_data, other.m_data, size * sizeof(T), hipMemcpyDeviceToDevice));
	}
	void copy_from_device(const GPUMemory<T>& other) { copy_from_device(other, other.m_size); }
	GPUMemory<T> copy(size_t size) const {
		GPUMemory<T> r{size};
		HIP_CHECK_THROW(hipMemcpy(r.m_data, m_data, size * sizeof(T), hipMemcpyDeviceToDevice));
		return r;
	}
	GPUMemory<T> copy() const { return copy(m_size); }

	T* data() const { return m_data; }
	bool managed() const { return m_managed; }
	size_t get_num_elements() const { return m_size; }
	size_t size() const { return m_size; }
	size_t get_bytes() const { return m_size * sizeof(T); }
	size_t bytes() const { return get_bytes(); }

private:
	T* m_data = nullptr;
	size_t m_size = 0;
	bool m_managed = false;
};

// gpu_memory.h:426-754
class GPUMemoryArena {
public:
	// a workspace interval of one stream's arena, returned to it on destruction (move-only)
	class Allocation {
	public:
		Allocation() = default;
		Allocation(hipStream_t stream, uint8_t* data) : m_stream{stream}, m_data{data} {}
		~Allocation() {
			if (m_data) tcnn_workspace_free(m_stream, m_data);
		}
		Allocation(const Allocation&) = delete;
		Allocation& operator=(const Allocation&) = delete;
		Allocation(Allocation&& other) { *this = std::move(other); }
		Allocation& operator=(Allocation&& other) {
			std::swap(m_stream, other.m_stream);
			std::swap(m_data, other.m_data);
			return *this;
		}
		uint8_t* data() { return m_data; }
		const uint8_t* data() const { return m_data; }
		hipStream_t stream() const { return m_stream; }

	private:
		hipStream_t m_stream = nullptr;
		uint8_t* m_data = nullptr;
	};
};

inline size_t align_to_cacheline(size_t bytes) { return (bytes + 127) / 128 * 128; }

inline GPUMemoryArena::Allocation allocate_workspace(hipStream_t stream, size_t n_bytes) {
	if (n_bytes == 0) return {};
	void* p = tcnn_workspace_allocate(stream, n_bytes);
	if (!p) throw std::runtime_error{tcnn_last_error()};
	return GPUMemoryArena::Allocation{stream, (uint8_t*)p};
}

// one allocation split into cache-line aligned arrays (gpu_memory.h:726-741)
namespace detail {
template <typename... Types, size_t... I>
std::tuple<Types*...> distribute(uint8_t* base, std::index_sequence<I...>, const size_t (&offsets)[sizeof...(Types)]) {
	return std::tuple<Types*...>{(Types*)(base + offsets[I])...};
}
}  // namespace detail

template <typename... Types, typename... Sizes>
std::tuple<Types*...> allocate_workspace_and_distribute(hipStream_t stream, GPUMemoryArena::Allocation* alloc, Sizes... sizes) {
	static_assert(sizeof...(Types) == sizeof...(Sizes), "allocate_workspace_and_distribute: one size per type");
	const size_t bytes[] = {align_to_cacheline((size_t)sizes * sizeof(Types))...};
	size_t offsets[sizeof...(Types)];
	size_t total = 0;
	for (size_t i = 0; i < sizeof...(Types); ++i) {
		offsets[i] = total;
		total += bytes[i];
	}
	*alloc = allocate_workspace(stream, total);
	return detail::distribute<Types...>(alloc->data(), std::index_sequence_for<Types...>{}, offsets);
}

// gpu_memory.h:743-754: drops the stream's arena (it must hold no live allocation)
inline void free_gpu_memory_arena(hipStream_t stream) {
	if (tcnn_free_workspace_arena(stream) != 0) throw std::runtime_error{tcnn_last_error()};
}

}  // namespace tcnn
