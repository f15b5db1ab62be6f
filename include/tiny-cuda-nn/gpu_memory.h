// tiny-cuda-nn/gpu_memory.h -- GPUMemory<T> (reference include/tiny-cuda-nn/gpu_memory.h:60-390):
// an owning, move-only device array. The engine's own temporaries live in its workspaces (grow-only,
// address-stable across steps), so the reference's stream arenas (gpu_memory.h:426-754) have no
// counterpart here beyond free_all_gpu_memory_arenas() (common.h).
#pragma once

#include <cstring>
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

}  // namespace tcnn
