// tiny-cuda-nn/gpu_matrix.h -- GPUMatrixDynamic<T> / GPUMatrix<T, layout> (reference
// include/tiny-cuda-nn/gpu_matrix.h:105-480): m() rows = features, n() columns = batch; ColumnMajor
// (the default) stores element (i, j) at data[i + j * m], i.e. one sample's features contiguous --
// exactly the [n x n_features] sample-major buffers the engine's C-ABI takes.
#pragma once

#include <memory>
#include <vector>

#include "gpu_memory.h"

namespace tcnn {

template <typename T>
class GPUMatrixDynamic {
public:
	using Type = T;

	GPUMatrixDynamic() = default;
	// owning (gpu_matrix.h:117-125); the stream argument of the reference's arena overload is accepted
	GPUMatrixDynamic(uint32_t m, uint32_t n, MatrixLayout layout = CM) : m_rows{m}, m_cols{n}, m_layout{layout} {
		m_owned = std::make_shared<GPUMemory<T>>((size_t)m * n);
		m_data = m_owned->data();
	}
	GPUMatrixDynamic(uint32_t m, uint32_t n, hipStream_t, MatrixLayout layout = CM) : GPUMatrixDynamic(m, n, layout) {}
	// non-owning view of caller memory (gpu_matrix.h:127-130)
	GPUMatrixDynamic(T* data, uint32_t m, uint32_t n, MatrixLayout layout = CM, uint32_t stride = 0)
	    : m_data{data}, m_rows{m}, m_cols{n}, m_layout{layout}, m_stride{stride} {}

	GPUMatrixDynamic(GPUMatrixDynamic<T>&& other) = default;
	GPUMatrixDynamic<T>& operator=(GPUMatrixDynamic<T>&& other) = default;
	GPUMatrixDynamic(const GPUMatrixDynamic<T>&) = delete;
	GPUMatrixDynamic<T>& operator=(const GPUMatrixDynamic<T>&) = delete;
	virtual ~GPUMatrixDynamic() = default;

	T* data() const { return m_data; }
	uint32_t m() const { return m_rows; }
	uint32_t n() const { return m_cols; }
	uint32_t rows() const { return m_rows; }
	uint32_t cols() const { return m_cols; }
	uint32_t stride() const { return m_stride ? m_stride : (m_layout == CM ? m_rows : m_cols); }
	MatrixLayout layout() const { return m_layout; }
	size_t n_elements() const { return (size_t)m_rows * m_cols; }
	size_t n_bytes() const { return n_elements() * sizeof(T); }
	bool is_contiguous() const { return stride() == (m_layout == CM ? m_rows : m_cols); }

	// gpu_matrix.h:226-233
	GPUMatrixDynamic<T> transposed() const {
		return GPUMatrixDynamic<T>(m_data, m_cols, m_rows, m_layout == CM ? RM : CM, stride());
	}
	GPUMatrixDynamic<T> view() const { return GPUMatrixDynamic<T>(m_data, m_rows, m_cols, m_layout, stride()); }

	void memset(int value) {
		CHECK_THROW(is_contiguous());
		HIP_CHECK_THROW(hipMemset(m_data, value, n_bytes()));
	}
	void memset_async(hipStream_t stream, int value) {
		CHECK_THROW(is_contiguous());
		HIP_CHECK_THROW(hipMemsetAsync(m_data, value, n_bytes(), stream));
	}

	std::vector<T> to_cpu_vector() const {
		CHECK_THROW(is_contiguous());
		std::vector<T> v(n_elements());
		HIP_CHECK_THROW(hipMemcpy(v.data(), m_data, n_bytes(), hipMemcpyDeviceToHost));
		return v;
	}

protected:
	T* m_data = nullptr;
	uint32_t m_rows = 0, m_cols = 0;
	MatrixLayout m_layout = CM;
	uint32_t m_stride = 0;
	std::shared_ptr<GPUMemory<T>> m_owned;
};

template <typename T, MatrixLayout _layout = MatrixLayout::ColumnMajor>
class GPUMatrix : public GPUMatrixDynamic<T> {
public:
	static constexpr MatrixLayout static_layout = _layout;
	static constexpr MatrixLayout static_transposed_layout = _layout == RM ? CM : RM;

	GPUMatrix() : GPUMatrixDynamic<T>{nullptr, 0, 0, static_layout} {}
	GPUMatrix(uint32_t m, uint32_t n) : GPUMatrixDynamic<T>{m, n, static_layout} {}
	GPUMatrix(uint32_t m, uint32_t n, hipStream_t stream) : GPUMatrixDynamic<T>{m, n, stream, static_layout} {}
	GPUMatrix(T* data, uint32_t m, uint32_t n, uint32_t stride = 0) : GPUMatrixDynamic<T>{data, m, n, static_layout, stride} {}
	GPUMatrix(GPUMatrix<T, static_layout>&& other) = default;
	GPUMatrix<T, static_layout>& operator=(GPUMatrix<T, static_layout>&& other) = default;
	GPUMatrix(const GPUMatrix<T, static_layout>&) = delete;
	GPUMatrix<T, static_layout>& operator=(const GPUMatrix<T, static_layout>&) = delete;

	GPUMatrix<T, static_transposed_layout> transposed() const {
		return GPUMatrix<T, static_transposed_layout>(this->data(), this->n(), this->m(), this->stride());
	}
};

template <typename T>
using GPUMatrixRM = GPUMatrix<T, RM>;
template <typename T>
using GPUMatrixCM = GPUMatrix<T, CM>;

}  // namespace tcnn
