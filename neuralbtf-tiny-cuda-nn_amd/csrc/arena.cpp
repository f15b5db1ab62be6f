// arena.cpp -- stream-ordered workspace arena (reference include/tiny-cuda-nn/gpu_memory.h:426-754:
// GPUMemoryArena, allocate_workspace, free_gpu_memory_arena), behind the C-ABI tcnn_workspace_*.
//
// One arena per stream (per device for the null stream). The arena reserves one virtual address
// range the size of the device's memory (hipMemAddressReserve) and maps physical memory at its end
// as it grows (hipMemCreate / hipMemMap / hipMemSetAccess), so an allocation's address never moves
// when the arena grows -- the property that lets captured hipGraphs keep their pointers. Without
// virtual memory management it falls back to one hipMalloc'd buffer that is re-allocated (and
// copied) 1.5x larger, as the reference's fallback does. Allocations are 128-byte aligned
// intervals, first fit, freed intervals merged.
//
// Lifetime as the reference's shared_ptr<GPUMemoryArena> (gpu_memory.h:690-760): free_gpu_memory_arena
// and free_all_gpu_memory_arenas detach arenas from their streams; a detached arena lives on until its
// last allocation is freed. An arena is built on the device its stream belongs to. Growth never
// synchronises on the VMM path (mapping is complete when hipMemSetAccess returns, and queued work
// cannot touch the new range), so allocating while a stream is being captured is legal there; the
// fallback's copy-to-a-larger-buffer needs the device idle and refuses under capture.
#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "runtime.h"

namespace tcnn_amd {

namespace {

constexpr size_t ARENA_ALIGN = 128;

struct Arena {
	int device = 0;
	bool vmm = false;
	char* base = nullptr;       // VMM: reserved range; fallback: the buffer
	size_t max_size = 0, size = 0, gran = 1;
	std::vector<hipMemGenericAllocationHandle_t> handles;
	std::vector<std::pair<size_t, size_t>> mapped;  // (offset, bytes) of each mapped chunk
	std::map<size_t, size_t> free_iv;               // start -> end
	std::unordered_map<size_t, size_t> used;        // start -> bytes
	std::vector<void*> old_bufs;                    // fallback: earlier buffers, kept for live pointers
	std::unordered_map<const void*, size_t> offset_of;  // live pointer -> interval start

	explicit Arena(int dev) : device(dev) {
		int vm = 0;
		hipDeviceGetAttribute(&vm, hipDeviceAttributeVirtualMemoryManagementSupported, device);
		size_t free_b = 0, total_b = 0;
		TCNN_HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
		hipMemAllocationProp prop = {};
		prop.type = hipMemAllocationTypePinned;
		prop.location.type = hipMemLocationTypeDevice;
		prop.location.id = device;
		// chunks of the recommended granularity and at least 2 MiB, so every mapped chunk starts on a
		// 2 MiB boundary of the range (the minimum, 4 KiB, mapped and accessed fine for small chunks
		// but hipMemSetAccess refused a 3 GiB chunk mapped at a 4 KiB offset)
		if (vm && hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended) == hipSuccess && gran > 0) {
			gran = std::max<size_t>(gran, (size_t)2 << 20);
			max_size = total_b / gran * gran;
			void* p = nullptr;
			if (hipMemAddressReserve(&p, max_size, 0, nullptr, 0) == hipSuccess) {
				base = (char*)p;
				vmm = true;
			}
		}
		if (!vmm) {
			gran = 1u << 21;
			max_size = total_b;
		}
		free_iv[0] = max_size;
	}
	~Arena() {
		// queued work may still use the memory (the reference frees with the same caveat); an arena is
		// destroyed only when detached and empty, never under capture
		int cur = 0;
		hipGetDevice(&cur);
		hipSetDevice(device);
		hipDeviceSynchronize();
		if (vmm) {
			for (auto& m : mapped) hipMemUnmap(base + m.first, m.second);
			for (auto h : handles) hipMemRelease(h);
			if (base) hipMemAddressFree(base, max_size);
		} else {
			if (base) hipFree(base);
			for (void* b : old_bufs) hipFree(b);
		}
		hipSetDevice(cur);
	}
	bool in_use() const { return !used.empty(); }

	void enlarge(size_t n_bytes, hipStream_t st) {  // gpu_memory.h:510-601
		if (n_bytes <= size) return;
		if (!vmm) {
			hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
			if (st) TCNN_HIP_CHECK(hipStreamIsCapturing(st, &cs));
			TCNN_CHECK(cs == hipStreamCaptureStatusNone,
			           "GPUMemoryArena: growing the fallback arena (no virtual memory support) under stream capture");
			TCNN_HIP_CHECK(hipDeviceSynchronize());  // queued work may still read the old buffer
			const size_t ns = (size_t)(n_bytes * 1.5 + gran - 1) / gran * gran;
			void* p = nullptr;
			TCNN_HIP_CHECK(hipMalloc(&p, ns));
			if (base) {  // live allocations keep pointing at the old buffer (freed with the arena)
				TCNN_HIP_CHECK(hipMemcpy(p, base, size, hipMemcpyDeviceToDevice));
				old_bufs.push_back(base);
			}
			base = (char*)p;
			size = ns;
			return;
		}
		const size_t add = (n_bytes - size + gran - 1) / gran * gran;
		// mapped as chunks of at most MAX_CHUNK (a chunk whose map or access fails is retried as
		// granularity-sized pieces); `size` advances with every mapped piece, so a failure part-way
		// leaves the arena consistent (the mapped prefix is kept and reused by the next growth)
		constexpr size_t MAX_CHUNK = (size_t)256 << 20;
		const size_t target = size + add;
		while (size < target) {
			const size_t want = std::min(MAX_CHUNK, target - size);
			if (map_chunk(size, want)) {
				size += want;
				continue;
			}
			for (size_t o = 0; o < want; o += gran) {
				if (!map_chunk(size, gran)) throw std::runtime_error("GPUMemoryArena: mapping device memory failed");
				size += gran;
			}
		}
	}

	bool map_chunk(size_t off, size_t bytes) {
		hipMemAllocationProp prop = {};
		prop.type = hipMemAllocationTypePinned;
		prop.location.type = hipMemLocationTypeDevice;
		prop.location.id = device;
		hipMemGenericAllocationHandle_t h;
		if (hipMemCreate(&h, bytes, &prop, 0) != hipSuccess) return false;
		if (hipMemMap(base + off, bytes, 0, h, 0) != hipSuccess) {
			hipMemRelease(h);
			return false;
		}
		hipMemAccessDesc acc = {};
		acc.location.type = hipMemLocationTypeDevice;
		acc.location.id = device;
		acc.flags = hipMemAccessFlagsProtReadWrite;
		if (hipMemSetAccess(base + off, bytes, &acc, 1) != hipSuccess) {
			hipMemUnmap(base + off, bytes);
			hipMemRelease(h);
			hipGetLastError();
			return false;
		}
		handles.push_back(h);
		mapped.emplace_back(off, bytes);
		return true;
	}

	size_t allocate(size_t n, hipStream_t st) {  // gpu_memory.h:563-592: first fit
		n = std::max<size_t>((n + ARENA_ALIGN - 1) / ARENA_ALIGN * ARENA_ALIGN, ARENA_ALIGN);
		for (auto it = free_iv.begin(); it != free_iv.end(); ++it) {
			if (it->second - it->first < n) continue;
			const size_t start = it->first, end = it->second;
			enlarge(start + n, st);  // may throw: the interval lists are untouched until it succeeded
			free_iv.erase(it);
			if (start + n < end) free_iv[start + n] = end;
			used[start] = n;
			return start;
		}
		throw std::runtime_error("GPUMemoryArena: out of memory");
	}

	void release(size_t start) {  // gpu_memory.h:594-611: free + merge adjacent intervals
		auto u = used.find(start);
		TCNN_CHECK(u != used.end(), "GPUMemoryArena: freeing an address that was not allocated");
		size_t s = start, e = start + u->second;
		used.erase(u);
		auto next = free_iv.lower_bound(s);
		if (next != free_iv.end() && next->first == e) {
			e = next->second;
			next = free_iv.erase(next);
		}
		if (next != free_iv.begin()) {
			auto prev = std::prev(next);
			if (prev->second == s) {
				s = prev->first;
				free_iv.erase(prev);
			}
		}
		free_iv[s] = e;
	}
};

struct Arenas {
	std::mutex mu;
	std::unordered_map<hipStream_t, std::shared_ptr<Arena>> by_stream;
	std::unordered_map<int, std::shared_ptr<Arena>> by_device;  // the null stream
	std::unordered_map<const void*, std::shared_ptr<Arena>> owner;  // live allocation -> its arena
	std::shared_ptr<Arena>& get(hipStream_t st) {
		if (st) {
			auto& a = by_stream[st];
			if (!a) {
				int dev = 0;
				TCNN_HIP_CHECK(hipStreamGetDevice(st, &dev));  // the stream's device, not the current one
				a = std::make_shared<Arena>(dev);
			}
			return a;
		}
		int d = 0;
		TCNN_HIP_CHECK(hipGetDevice(&d));
		auto& a = by_device[d];
		if (!a) a = std::make_shared<Arena>(d);
		return a;
	}
};

Arenas& arenas() {
	static Arenas* a = new Arenas;  // never destroyed: arenas may outlive static destruction order
	return *a;
}

}  // namespace

void* workspace_allocate(hipStream_t st, size_t n_bytes) {
	if (n_bytes == 0) return nullptr;
	Arenas& A = arenas();
	std::lock_guard<std::mutex> lk(A.mu);
	std::shared_ptr<Arena> a = A.get(st);
	int cur = 0;
	TCNN_HIP_CHECK(hipGetDevice(&cur));
	if (cur != a->device) TCNN_HIP_CHECK(hipSetDevice(a->device));
	size_t off = 0;
	try {
		off = a->allocate(n_bytes, st);
	} catch (...) {
		if (cur != a->device) hipSetDevice(cur);
		throw;
	}
	if (cur != a->device) TCNN_HIP_CHECK(hipSetDevice(cur));
	void* p = a->base + off;
	a->offset_of[p] = off;
	A.owner[p] = a;
	return p;
}

void workspace_free(hipStream_t st, void* p) {
	(void)st;  // the allocation knows its arena (which may have been detached from the stream since)
	if (!p) return;
	Arenas& A = arenas();
	std::shared_ptr<Arena> a;
	{
		std::lock_guard<std::mutex> lk(A.mu);
		auto o = A.owner.find(p);
		TCNN_CHECK(o != A.owner.end(), "GPUMemoryArena: freeing an address that no arena allocated");
		a = std::move(o->second);
		A.owner.erase(o);
		auto it = a->offset_of.find(p);
		a->release(it->second);
		a->offset_of.erase(it);
	}
	// `a` going out of scope here destroys a detached arena whose last allocation this was
}

// free_gpu_memory_arena (gpu_memory.h:743-749): detach the stream's arena; it is destroyed now if it
// has no live allocations, else when its last one is freed
void workspace_arena_free(hipStream_t st) {
	Arenas& A = arenas();
	std::shared_ptr<Arena> drop;
	{
		std::lock_guard<std::mutex> lk(A.mu);
		if (st) {
			auto it = A.by_stream.find(st);
			if (it == A.by_stream.end()) return;
			drop = std::move(it->second);
			A.by_stream.erase(it);
		} else {
			int d = 0;
			TCNN_HIP_CHECK(hipGetDevice(&d));
			auto it = A.by_device.find(d);
			if (it == A.by_device.end()) return;
			drop = std::move(it->second);
			A.by_device.erase(it);
		}
	}
}

// free_all_gpu_memory_arenas (gpu_memory.h:751-754)
void workspace_arena_free_all() {
	Arenas& A = arenas();
	std::vector<std::shared_ptr<Arena>> drop;
	{
		std::lock_guard<std::mutex> lk(A.mu);
		for (auto& kv : A.by_stream) drop.push_back(std::move(kv.second));
		for (auto& kv : A.by_device) drop.push_back(std::move(kv.second));
		A.by_stream.clear();
		A.by_device.clear();
	}
}

void workspace_arena_info(hipStream_t st, uint64_t* mapped_bytes, int* vmm) {
	Arenas& A = arenas();
	std::lock_guard<std::mutex> lk(A.mu);
	Arena& a = *A.get(st);
	if (mapped_bytes) *mapped_bytes = a.size;
	if (vmm) *vmm = a.vmm ? 1 : 0;
}

}  // namespace tcnn_amd
