// dp_peer.hip -- the data-parallel exchange over peer-mapped device memory (xGMI), without a
// collective library.
//
// Why: at 8 ranks a rank's step is 2^15 points (~48 us on one MI355X) while every RCCL collective
// costs ~28 us of latency (profiles/r03_dp_floor.json), so the RCCL schedules cannot scale. Here the
// ranks of a node exchange through each other's memory directly: every rank exports IPC handles of
// its gradient / parameter / optimizer-state buffers and a small flag array; after attaching, one
// training step is
//   local step (fused kernel, grid backward; the gradient sums complete in g32)
//   -> signal "gradients ready" (a monotonic per-rank counter in the rank's own flag array)
//   -> wait until every rank's counter reached this step (one workgroup polls; timeout guarded)
//   -> Adam on this rank's 1/N shard, reading the gradient of parameter i as
//      sum_p g32_p[i] over the ranks p = 0 .. N-1 in that fixed order (peer loads over xGMI)
//   -> signal "weights ready" -> wait -> copy the other ranks' updated fp16 shards into w16.
// Per rank and step that moves (N-1)/N of 4 + 2 bytes per parameter over the links -- the
// reduce-scatter + all-gather volume -- with no collective launch, no proxy thread and no host
// involvement; every kernel reads its step counter from device memory, so the step is also
// graph-capturable. The shards are summed in rank order on the rank that owns them, so replicas
// stay bit-identical (and, for two ranks, bit-identical to any all-reduce: a + b is one sum).
//
// Coherence without fences: everything another rank reads -- this rank's gradient sums, its updated
// fp16 shard, its optimizer-state shard when gathered, and the step counters -- lives in UNCACHED
// device memory (hipDeviceMallocUncached: every access goes to memory, as RCCL allocates its
// protocol buffers), written once and read once per step, so no L2 holds a stale copy and no
// acquire / release cache maintenance is needed (a first version used fine-grained-free buffers with
// a system-scope acquire per workgroup: 147 us per step on one rank, the repeated L2 invalidations).
// The parameters the kernels re-read (the grid table) stay in ordinary memory: the gather copies the
// peers' shards from their uncached mirrors into it. Kernel boundaries order the stores of one rank's
// stream; the counters are stored and polled with system-scope atomics.
//
// Waits are one-workgroup kernels of their own (the data kernels launch after them), so a waiting
// rank never occupies the CUs another rank on the same GPU needs to make progress (the 2-process
// test shares one GPU). Every wait gives up after a timeout, raising an error flag in host-mapped
// memory that the next step (or gather) turns into an exception -- a dead peer cannot hang the GPU.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "adam_device.h"
#include "runtime.h"

namespace tcnn_amd {

namespace {

constexpr uint32_t PEER_MAGIC = 0x50454552u;  // "PEER"
constexpr int PEER_MAX_RANKS = 64;  // one wave polls the ranks' counters
constexpr int PEER_NBUF = 4;                  // exported: gradient sums, fp16 shard mirror, state staging, counters
enum PeerBuf { PB_G32 = 0, PB_W16, PB_STATE, PB_FLAGS };
enum PeerSlot { SLOT_GRAD = 0, SLOT_WEIGHTS = 1, SLOT_GATHER = 2, SLOT_DETACH = 3, SLOT_PROBE = 4 };
constexpr int PROBE_WORD = 16;  // the attach probe's token in each rank's counter page

__host__ __device__ inline uint32_t probe_token(int rank) { return PEER_MAGIC ^ (0x9e3779b9u * (uint32_t)(rank + 1)); }
enum PeerCtr { CTR_STEP = 0, CTR_SYNC = 1, CTR_ERR = 2, CTR_ARRIVE = 3 };

struct PeerBlob {
	uint32_t magic, nranks, rank, device;
	uint64_t n_params, per;
	uint64_t pci;  // hash of the device's PCI bus id: ranks that share one GPU (the 1-GPU tests) see equal values
	hipIpcMemHandle_t h[PEER_NBUF];
};

__device__ __forceinline__ uint32_t load_sys(const uint32_t* p) {
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one workgroup: when my_flags != nullptr first signal -- counter ctr[c] (+1 when bump), then my_flags[slot]
// = that value (system-scope store; every earlier write of this stream went to uncached memory and
// finished with its kernel) -- then wait until every rank's flags[slot] reached ctr[c]; on timeout
// raise *err (host-mapped)
struct PeerFlags {  // the ranks' counter arrays, by value (no dependent pointer load before the polls)
	uint32_t* f[PEER_MAX_RANKS];
};
// ctr[CTR_ERR] is the device-side copy of the error flag: the step's data kernels read it and leave
// the parameters untouched once a wait has failed (the host-mapped *err raises at the next call)
__global__ void k_peer_wait(const PeerFlags fl, int nranks, int slot, uint32_t* __restrict__ ctr, int c, long long timeout_ticks,
                            int* __restrict__ err, uint32_t* __restrict__ my_flags, int bump) {
	if (threadIdx.x >= 64) return;
	if (ctr[CTR_ERR]) return;  // an earlier wait failed: no signal, no wait (the step is abandoned)
	uint32_t target = ctr[c];
	if (my_flags && threadIdx.x == 0) {
		if (bump) ctr[c] = target + 1u;
		__hip_atomic_store(my_flags + slot, target + (bump ? 1u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
	}
	if (my_flags && bump) target += 1u;
	// lane p polls rank p: the ranks' counters are read concurrently (one link round trip per poll, not N)
	const int p = threadIdx.x;
	const long long t0 = wall_clock64();
	for (;;) {
		const bool ok = p >= nranks || (int32_t)(load_sys(fl.f[p] + slot) - target) >= 0;
		const uint64_t pending = __builtin_amdgcn_ballot_w64(!ok);
		if (pending == 0) return;
		if (wall_clock64() - t0 > timeout_ticks) {
			if (p == (int)__builtin_ctzll(pending)) {
				__hip_atomic_store(err, 1 + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
				ctr[CTR_ERR] = 1u + (uint32_t)p;
			}
			return;
		}
		__builtin_amdgcn_s_sleep(1);
	}
}

// attach probe: this rank's token into its own counter page; after a barrier every rank reads every
// rank's token through the peer mappings (a mapping that does not reach the peer's memory shows up
// here, once, instead of as a step that never completes)
__global__ void k_peer_token(uint32_t* __restrict__ my_flags, uint32_t token) {
	if (threadIdx.x == 0) __hip_atomic_store(my_flags + PROBE_WORD, token, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_peer_probe(const PeerFlags fl, int nranks, int* __restrict__ err, uint32_t* __restrict__ ctr) {
	const int p = threadIdx.x;
	if (p < nranks && load_sys(fl.f[p] + PROBE_WORD) != probe_token(p)) {
		__hip_atomic_store(err, 1000 + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
		ctr[CTR_ERR] = 1000u + (uint32_t)p;
	}
}

// The poll of a step kernel's head, by wave 0 of every workgroup: lane p reads rank p's flags[slot]
// until every rank reached `target`. Returns false (and raises the error flags once) on a timeout.
__device__ __forceinline__ bool peer_poll(const PeerFlags& fl, int nranks, int slot, uint32_t target, long long timeout_ticks,
                                          int* __restrict__ err, uint32_t* __restrict__ ctr) {
	const int p = threadIdx.x;
	const long long t0 = wall_clock64();
	for (;;) {
		const bool ok = p >= nranks || (int32_t)(load_sys(fl.f[p] + slot) - target) >= 0;
		const uint64_t pending = __builtin_amdgcn_ballot_w64(!ok);
		if (pending == 0) return true;
		if (wall_clock64() - t0 > timeout_ticks) {
			if (p == (int)__builtin_ctzll(pending)) {
				__hip_atomic_store(err, 1 + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
				__hip_atomic_store(ctr + CTR_ERR, 1u + (uint32_t)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			}
			return false;
		}
		__builtin_amdgcn_s_sleep(1);
	}
}

struct PeerStepArgs {
	PeerFlags fl;
	const float* g[PEER_MAX_RANKS];  // the ranks' gradient-sum mirrors, by value (no pointer-table load)
	_Float16* w16_mirror;            // this rank's fp16 shard mirror (the peers gather from it)
	uint32_t* ctr;                   // this rank's local counters
	uint32_t* my_flags;              // this rank's exported counter page
	int* err;                        // host-mapped error flag
	long long timeout_ticks;
	int nranks;
	int signal;  // 1: signal "gradients ready" here (every workgroup; the previous launches' stores completed)
};

// arrival of a workgroup whose stores the signal covers: every storing wave's vmcnt(0) wait, the
// barrier, then one agent-scope add; returns true in the last-arriving workgroup's thread 0. What
// the peers read is in UNCACHED memory (no L2 holds it), so completed stores are visible -- no release
// fence (an agent- or system-scope one writes back the XCD's whole L2, ~2-7 us, for stores nobody
// else reads)
__device__ __forceinline__ bool peer_arrive(uint32_t* __restrict__ ctr, int slot_ctr) {
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	if (threadIdx.x != 0) return false;
	const uint32_t prev = __hip_atomic_fetch_add(ctr + slot_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	if (prev != gridDim.x * gridDim.y * gridDim.z - 1u) return false;
	__hip_atomic_store(ctr + slot_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	return true;
}

// One launch for "wait for every rank's gradients -> sharded Adam -> weights ready" (r06; r05 ran a
// one-workgroup wait kernel before and after Adam). Every workgroup reads the step number s + 1 from
// ctr[CTR_STEP] (signalling this rank's gradients itself when the previous launch did not: the same
// idempotent system-scope store from every workgroup), issues the Adam-state loads of its first
// parameter group, waits for every rank's signal, runs Adam on its part of this rank's shard
// [a.begin, a.n) -- 4 parameters per thread, the gradient of parameter i summed over the ranks'
// mirrors in rank order g_0 + g_1 + ... -- writes the updated fp16 values to its mirror, and arrives
// on ctr[CTR_ARRIVE]. The last arrival (every workgroup has read ctr[CTR_STEP] by then) bumps
// ctr[CTR_STEP] and signals "weights ready" for the gather. Workgroups wait only on other ranks,
// never on each other, so co-residency is not needed.
__global__ __launch_bounds__(256) void k_peer_adam(const AdamArgs a, const AdamBuffers s, const PeerStepArgs pa) {
	__shared__ int ok_s;
	const uint32_t step = pa.ctr[CTR_STEP] + 1u;
	const uint32_t stride = gridDim.x * blockDim.x * 4;
	const uint32_t i0 = a.begin + (blockIdx.x * blockDim.x + threadIdx.x) * 4;
	AdamState4 st0{};
	if (i0 + 4 <= a.n) st0 = adam_load4(s, i0);  // local state: in flight across the wait
	if (threadIdx.x < 64) {
		bool ok = pa.ctr[CTR_ERR] == 0u;  // an earlier wait failed: no signal, no wait (the step is abandoned)
		if (ok && pa.signal && threadIdx.x == 0) {
			__hip_atomic_store(pa.my_flags + SLOT_GRAD, step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // landed before this wave's first poll reads it back
		}
		if (ok) ok = peer_poll(pa.fl, pa.nranks, SLOT_GRAD, step, pa.timeout_ticks, pa.err, pa.ctr);
		if (threadIdx.x == 0) ok_s = ok;
	}
	__syncthreads();
	if (ok_s) {
		for (uint32_t i = i0; i < a.n; i += stride) {
			if (i + 4 <= a.n) {
				f4 g = *(const f4*)(pa.g[0] + i);
				for (int p0 = 1; p0 < pa.nranks; p0 += 8) {  // loads in flight together, additions in rank order
					f4 v[8];
#pragma unroll
					for (int u = 0; u < 8; ++u)
						if (p0 + u < pa.nranks) v[u] = *(const f4*)(pa.g[p0 + u] + i);
#pragma unroll
					for (int u = 0; u < 8; ++u)
						if (p0 + u < pa.nranks) g += v[u];
				}
				*(f4*)(s.g32 + i) = g;
				const float gs[4] = {g.x, g.y, g.z, g.w};
				const AdamState4 st = i == i0 ? st0 : adam_load4(s, i);
				adam_store4(a, s, i, gs, st);
				*(h4*)(pa.w16_mirror + i) = *(const h4*)(s.w16 + i);
			} else {
				for (uint32_t k = i; k < a.n; ++k) {
					float g = pa.g[0][k];
					for (int p = 1; p < pa.nranks; ++p) g += pa.g[p][k];
					s.g32[k] = g;
					pa.w16_mirror[k] = adam_update(a, s, k, g);
				}
			}
		}
	}
	if (peer_arrive(pa.ctr, CTR_ARRIVE)) {  // the last arrival: every workgroup's mirror stores completed
		__hip_atomic_store(pa.ctr + CTR_STEP, step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (__hip_atomic_load(pa.ctr + CTR_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
			__hip_atomic_store(pa.my_flags + SLOT_WEIGHTS, step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
	}
}

// copy every other rank's shard of up to 4 buffers (blockIdx.z) from its mirror into the local
// arrays; blockIdx.y = the rank copied from (its mirror pointer a kernel argument), 16 bytes per
// thread in a grid-stride loop; shard bytes are multiples of 16. With poll != 0 (the training step)
// wave 0 of every workgroup first waits until every rank signalled "weights ready" for step
// ctr[CTR_STEP] (r06: was a one-workgroup wait kernel of its own).
struct PeerGatherArgs {
	uint8_t* local[4];
	const uint8_t* peer[PEER_MAX_RANKS];  // the ranks' mirror (fp16 shard mirror or state staging) base
	uint64_t peer_offset[4];              // byte offset of buffer z inside each mirror
	uint32_t elem_bytes[4];
	uint32_t nranks, rank;
	uint64_t per;  // elements per shard
	uint32_t* ctr;  // CTR_ERR set: the peers' mirrors are not this step's, copy nothing
	PeerFlags fl;
	int* err;
	long long timeout_ticks;
	int poll;
};
__global__ __launch_bounds__(256) void k_peer_gather(const PeerGatherArgs g) {
	__shared__ int ok_s;
	const uint32_t p = blockIdx.y, b = blockIdx.z;
	if (p == g.rank) return;
	if (g.poll) {
		if (threadIdx.x < 64) {
			bool ok = g.ctr[CTR_ERR] == 0u;
			if (ok) ok = peer_poll(g.fl, (int)g.nranks, SLOT_WEIGHTS, g.ctr[CTR_STEP], g.timeout_ticks, g.err, g.ctr);
			if (threadIdx.x == 0) ok_s = ok;
		}
		__syncthreads();
		if (!ok_s) return;
	} else if (g.ctr[CTR_ERR]) {
		return;
	}
	const uint64_t shard_bytes = g.per * g.elem_bytes[b];
	const uint64_t units = shard_bytes / 16;
	const uint8_t* src = g.peer[p] + g.peer_offset[b] + p * shard_bytes;
	uint8_t* dst = g.local[b] + p * shard_bytes;
	for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < units; q += (uint64_t)gridDim.x * blockDim.x)
		*(uint4*)(dst + q * 16) = *(const uint4*)(src + q * 16);
}

// this rank's shard of the optimizer state into its uncached staging mirror (for the peers' gather)
__global__ __launch_bounds__(256) void k_peer_stage(const float* __restrict__ w32, const float* __restrict__ m1, const float* __restrict__ m2,
                                                    const uint32_t* __restrict__ steps, uint32_t* __restrict__ stage, uint64_t lo,
                                                    uint64_t cnt, uint64_t stride, const uint32_t* __restrict__ ctr) {
	if (ctr[CTR_ERR]) return;
	const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= cnt) return;
	const uint64_t i = lo + k;
	stage[i] = __float_as_uint(w32[i]);
	stage[stride + i] = __float_as_uint(m1[i]);
	stage[2 * stride + i] = __float_as_uint(m2[i]);
	stage[3 * stride + i] = steps[i];
}

}  // namespace

struct TrainerHost::PeerDp {
	int nranks = 1, rank = 0;
	uint64_t per = 0;
	bool attached = false;
	DevBuf ctr;    // [2] local counters (step, sync)
	DevBuf ptrs;   // [PEER_NBUF][nranks] device pointers (local ones for this rank)
	// uncached, exported: gradient sums [N*per] fp32, fp16 shard mirror [N*per], state staging
	// [4][N*per] (w32, m1, m2, steps), counters [64] uint32
	void* x[PEER_NBUF] = {nullptr, nullptr, nullptr, nullptr};
	std::vector<void*> opened;  // IPC mappings of the peers' buffers
	std::vector<void*> host_ptr;  // [PEER_NBUF][nranks] the same pointers as `ptrs`, host copy (kernel arguments)
	int* err_host = nullptr;
	int* err_dev = nullptr;
	long long timeout_ticks = 0;
	int clock_khz = 1;  // wall_clock64 rate
	PeerFlags flags_arg{};  // the ranks' counter arrays (k_peer_wait's argument)
	// another rank runs on this rank's GPU (time-shared tests and rehearsals): the step kernels that
	// poll other ranks then keep to a few workgroups, so their spinning waves leave the other ranks'
	// kernels the CUs they need (a 1024-thread grid-backward workgroup needs a whole CU's registers)
	bool shared_device = false;
	PeerDp() = default;
	~PeerDp() {
		// this rank's kernels may still read the peers' mappings (an asynchronous step just issued):
		// finish them before unmapping (the collective part -- peers done reading OUR mirrors -- is
		// dp_peer_detach's SLOT_DETACH wait)
		(void)hipDeviceSynchronize();
		for (void* p : opened) (void)hipIpcCloseMemHandle(p);
		for (void* p : x)
			if (p) (void)hipFree(p);
		if (err_host) (void)hipHostFree(err_host);
	}
	template <typename T>
	T* const* table(int b) const { return (T* const*)(ptrs.as<void*>() + (size_t)b * nranks); }
	void check() const {
		const int e = err_host ? *(volatile int*)err_host : 0;
		if (e >= 1000)
			throw std::runtime_error("data-parallel peer exchange: rank " + std::to_string(e - 1000) +
			                         "'s memory is not readable through its mapping (attach probe)");
		if (e)
			throw std::runtime_error("data-parallel peer exchange: rank " + std::to_string(e - 1) +
			                         " did not arrive within the timeout (a rank stopped, or the ranks' steps diverged)");
	}
};

uint64_t dp_peer_blob_bytes() { return sizeof(PeerBlob); }

// the peer waits' timeout (default TCNN_PEER_TIMEOUT_S or 300 s -- long enough for rank-0-only work
// between steps such as a snapshot or a render; RCCL's own default is 30 min); applies to the current
// attachment too
void TrainerHost::dp_peer_set_timeout(double seconds) {
	TCNN_CHECK(seconds > 0.0, "peer exchange: the timeout must be positive");
	peer_timeout_s = seconds;
	if (peer) peer->timeout_ticks = (long long)((double)peer->clock_khz * 1000.0 * seconds);
	if (graph) set_graph(use_graph);  // captured peer steps carry the old timeout as a kernel argument
}

void TrainerHost::peer_check() const {
	if (peer) peer->check();
}

double peer_default_timeout_s() {
	const char* e = std::getenv("TCNN_PEER_TIMEOUT_S");
	const double v = e ? std::atof(e) : 0.0;
	return v > 0.0 ? v : 300.0;
}

static void grow_keep(DevBuf& b, size_t bytes, size_t valid) {
	if (b.bytes >= bytes) return;
	DevBuf n;
	n.reserve(bytes);
	TCNN_HIP_CHECK(hipMemset(n.p, 0, bytes));
	if (b.p && valid) TCNN_HIP_CHECK(hipMemcpy(n.p, b.p, valid, hipMemcpyDeviceToDevice));
	std::swap(b.p, n.p);
	std::swap(b.bytes, n.bytes);
}

void TrainerHost::dp_peer_export(int nranks, int rank, void* blob_out) {
	TCNN_CHECK(!dp, "peer exchange: detach the RCCL communicator first (set_dp(NULL))");
	TCNN_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "peer exchange: rank outside [0, nranks)");
	TCNN_CHECK(nranks <= PEER_MAX_RANKS, "peer exchange: at most 64 ranks (the ranks of one node)");
	if (peer) dp_peer_detach();
	TCNN_HIP_CHECK(hipDeviceSynchronize());
	auto pd = std::make_shared<PeerDp>();
	pd->nranks = nranks;
	pd->rank = rank;
	// shards of a multiple of 8 parameters: 16-byte units of fp16 and fp32 shards alike
	const uint64_t per = ((n_params + nranks - 1) / nranks + 7) / 8 * 8;
	pd->per = per;
	const size_t pad = (size_t)(per * nranks);
	grow_keep(w32, pad * 4, n_params * 4);
	grow_keep(w16, pad * 2, n_params * 2);
	grow_keep(g16, pad * 2, n_params * 2);
	grow_keep(g32, pad * 4, n_params * 4);
	grow_keep(m1, pad * 4, n_params * 4);
	grow_keep(m2, pad * 4, n_params * 4);
	grow_keep(steps, pad * 4, n_params * 4);
	const size_t xbytes[PEER_NBUF] = {pad * 4, pad * 2, 4 * pad * 4, 256};
	for (int k = 0; k < PEER_NBUF; ++k) {
		TCNN_HIP_CHECK(hipExtMallocWithFlags(&pd->x[k], xbytes[k], hipDeviceMallocUncached));
		TCNN_HIP_CHECK(hipMemset(pd->x[k], 0, xbytes[k]));
	}
	pd->ctr.reserve(64);
	TCNN_HIP_CHECK(hipMemset(pd->ctr.p, 0, 64));
	TCNN_HIP_CHECK(hipHostMalloc((void**)&pd->err_host, 64, hipHostMallocMapped));
	*pd->err_host = 0;
	TCNN_HIP_CHECK(hipHostGetDevicePointer((void**)&pd->err_dev, pd->err_host, 0));
	int dev = 0, khz = 0;
	TCNN_HIP_CHECK(hipGetDevice(&dev));
	TCNN_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
	pd->clock_khz = std::max(khz, 1);
	pd->timeout_ticks = (long long)((double)pd->clock_khz * 1000.0 * peer_timeout_s);
	PeerBlob b;
	std::memset(&b, 0, sizeof(b));
	b.magic = PEER_MAGIC;
	b.nranks = (uint32_t)nranks;
	b.rank = (uint32_t)rank;
	b.device = (uint32_t)dev;
	b.n_params = n_params;
	b.per = per;
	{
		char bus[64] = {0};
		TCNN_HIP_CHECK(hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, dev));
		uint64_t h = 1469598103934665603ull;  // FNV-1a
		for (const char* c = bus; *c; ++c) h = (h ^ (uint64_t)(uint8_t)*c) * 1099511628211ull;
		b.pci = h;
	}
	for (int k = 0; k < PEER_NBUF; ++k) TCNN_HIP_CHECK(hipIpcGetMemHandle(&b.h[k], pd->x[k]));
	std::memcpy(blob_out, &b, sizeof(b));
	peer = std::move(pd);
	ws.wimage_valid = false;
}

void TrainerHost::dp_peer_attach(const void* blobs) {
	TCNN_CHECK(peer && !peer->attached, "peer exchange: export before attaching");
	PeerDp& pd = *peer;
	const int N = pd.nranks;
	std::vector<void*> host((size_t)PEER_NBUF * N);
	PeerBlob mine;
	std::memcpy(&mine, (const uint8_t*)blobs + (size_t)pd.rank * sizeof(PeerBlob), sizeof(mine));
	for (int p = 0; p < N; ++p) {
		PeerBlob b;
		std::memcpy(&b, (const uint8_t*)blobs + (size_t)p * sizeof(PeerBlob), sizeof(b));
		if (p != pd.rank && b.pci == mine.pci) pd.shared_device = true;
		TCNN_CHECK(b.magic == PEER_MAGIC && (int)b.nranks == N && (int)b.rank == p && b.n_params == n_params && b.per == pd.per,
		           "peer exchange: blob " + std::to_string(p) + " does not describe rank " + std::to_string(p) + " of the same model");
		for (int k = 0; k < PEER_NBUF; ++k) {
			if (p == pd.rank) {
				host[(size_t)k * N + p] = pd.x[k];
				continue;
			}
			void* q = nullptr;
			TCNN_HIP_CHECK(hipIpcOpenMemHandle(&q, b.h[k], hipIpcMemLazyEnablePeerAccess));
			pd.opened.push_back(q);
			host[(size_t)k * N + p] = q;
		}
	}
	for (int p = 0; p < N; ++p) pd.flags_arg.f[p] = (uint32_t*)host[(size_t)PB_FLAGS * N + p];
	pd.ptrs.reserve(host.size() * sizeof(void*));
	TCNN_HIP_CHECK(hipMemcpy(pd.ptrs.p, host.data(), host.size() * sizeof(void*), hipMemcpyHostToDevice));
	pd.host_ptr = host;
	// probe (collective): every rank's token readable through every mapping, checked once here so a
	// broken mapping fails the attach (and the caller falls back) instead of a step. The ranks reach this
	// point together (their blobs were just all-gathered): its wait -- also the first proof that the
	// peers' signals arrive through the mappings -- gives up after at most 30 s, not the step timeout
	hipLaunchKernelGGL(k_peer_token, dim3(1), dim3(64), 0, nullptr, (uint32_t*)pd.x[PB_FLAGS], probe_token(pd.rank));
	TCNN_HIP_CHECK(hipGetLastError());
	peer_wait(nullptr, CTR_SYNC, SLOT_PROBE, 1, std::min<long long>(pd.timeout_ticks, (long long)pd.clock_khz * 1000LL * 30));
	hipLaunchKernelGGL(k_peer_probe, dim3(1), dim3(64), 0, nullptr, pd.flags_arg, N, pd.err_dev, pd.ctr.as<uint32_t>());
	TCNN_HIP_CHECK(hipGetLastError());
	TCNN_HIP_CHECK(hipDeviceSynchronize());
	pd.check();
	pd.attached = true;
	peer_attached = true;
	peer_nranks = N;
	dp_sharded = true;
	dp_state_partial = false;
	dp_per = pd.per;
	grad_scale = grad_scale_user / (float)dp_nranks();
	if (graph) set_graph(use_graph);
}

// MEASUREMENT ONLY (debug_api.h tcnn_debug_peer_loopback): attach as rank 0 of `nranks` ranks whose
// buffers are all this rank's own, so one process runs exactly the per-rank kernels of an N-rank peer
// step -- Adam on a 1/N shard summing N mirrors, the gather of N - 1 shards, every poll -- without
// peers or links (the "other" shards it gathers are its own mirror's: the parameters it trains are
// meaningless; the time is what this rehearses).
void TrainerHost::dp_peer_loopback(int nranks) {
	std::vector<uint8_t> blob(sizeof(PeerBlob));
	dp_peer_export(nranks, 0, blob.data());
	PeerDp& pd = *peer;
	const int N = pd.nranks;
	std::vector<void*> host((size_t)PEER_NBUF * N);
	for (int k = 0; k < PEER_NBUF; ++k)
		for (int p = 0; p < N; ++p) host[(size_t)k * N + p] = pd.x[k];
	for (int p = 0; p < N; ++p) pd.flags_arg.f[p] = (uint32_t*)pd.x[PB_FLAGS];
	pd.ptrs.reserve(host.size() * sizeof(void*));
	TCNN_HIP_CHECK(hipMemcpy(pd.ptrs.p, host.data(), host.size() * sizeof(void*), hipMemcpyHostToDevice));
	pd.host_ptr = host;
	pd.attached = true;
	peer_attached = true;
	peer_nranks = N;
	dp_sharded = true;
	dp_state_partial = false;
	dp_per = pd.per;
	grad_scale = grad_scale_user / (float)dp_nranks();
	if (graph) set_graph(use_graph);
}

// wait for every rank's flags[slot] to reach counter c; with signal_bump >= 0 this rank signals first
// (bumping the counter when 1) in the same one-workgroup launch
void TrainerHost::peer_wait(hipStream_t st, int c, int slot, int signal_bump, long long timeout_ticks) {
	PeerDp& pd = *peer;
	hipLaunchKernelGGL(k_peer_wait, dim3(1), dim3(64), 0, st, pd.flags_arg, pd.nranks, slot, pd.ctr.as<uint32_t>(), c,
	                   timeout_ticks >= 0 ? timeout_ticks : pd.timeout_ticks,
	                   pd.err_dev, signal_bump >= 0 ? (uint32_t*)pd.x[PB_FLAGS] : nullptr, signal_bump > 0 ? 1 : 0);
	TCNN_HIP_CHECK(hipGetLastError());
}

void TrainerHost::training_step_peer(hipStream_t st, uint32_t B, const float* input, const float* target) {
	PeerDp& pd = *peer;
	pd.check();
	// this rank's gradient sums, straight into its uncached exchange buffer: the fused grid engine's
	// two-launch step, or any other engine's pass (tile, layer-wise) with its reductions writing there
	float* gx = (float*)pd.x[PB_G32];
	if (overlapped_ok()) {
		// (r06, tried: the slab reduction with the "gradients ready" signal from its last-arriving
		// workgroup, to take the signal's trip off k_peer_adam's head: 2,800 workgroups adding to one
		// counter serialise at ~88 adds / us -- 35 us)
		training_step_overlapped(st, B, input, target, false, gx);
	} else {
		mark(st, 0);
		model->fwd_bwd(st, ws, B, input, target, n_output_dims, loss_scale, w16.p, nullptr, nullptr, gx, [&](int ph) { mark(st, ph); });
		launch_sum(st, ws.loss_partial.as<float>(), ws.n_loss_partials, d_loss.as<float>());
		mark(st, 4);
	}
	const uint64_t lo = std::min<uint64_t>(n_params, (uint64_t)pd.rank * pd.per), hi = std::min<uint64_t>(n_params, lo + pd.per);
	++adam_step;
	AdamArgs a = adam_args_table(st, adam_step);
	a.begin = (uint32_t)lo;
	a.n = (uint32_t)hi;
	const AdamBuffers s{w32.as<float>(), w16.as<_Float16>(), g32.as<float>(), g16.as<_Float16>(), m1.as<float>(), m2.as<float>(),
	                    steps.as<uint32_t>()};
	PeerStepArgs pa{};
	pa.fl = pd.flags_arg;
	for (int p = 0; p < pd.nranks; ++p) pa.g[p] = (const float*)pd.host_ptr[(size_t)PB_G32 * pd.nranks + p];
	pa.w16_mirror = (_Float16*)pd.x[PB_W16];
	pa.ctr = pd.ctr.as<uint32_t>();
	pa.my_flags = (uint32_t*)pd.x[PB_FLAGS];
	pa.err = pd.err_dev;
	pa.timeout_ticks = pd.timeout_ticks;
	pa.nranks = pd.nranks;
	pa.signal = 1;
	// wait + Adam on this rank's shard + "weights ready", one launch (a rank with an empty shard still
	// launches one workgroup: it arrives and, last, signals)
	// at most 128 workgroups: each adds once to the arrival counter, and one word takes ~88 adds per us
	const uint32_t nwg = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(div_round_up(hi > lo ? hi - lo : 0, 1024), pd.shared_device ? 8 : 128));
	hipLaunchKernelGGL(k_peer_adam, dim3(nwg), dim3(256), 0, st, a, s, pa);
	TCNN_HIP_CHECK(hipGetLastError());
	peer_gather(st, 1, true);  // waits for every rank's "weights ready" in its head
	ws.wimage_valid = false;
	dp_state_partial = true;
	last_B = B;
}

// copy the other ranks' shards from their mirrors: what = 1: the fp16 parameters; 4: fp32 masters,
// both moments, step counts (from the staging mirror)
void TrainerHost::peer_gather(hipStream_t st, int what, bool poll) {
	PeerDp& pd = *peer;
	PeerGatherArgs g{};
	g.ctr = pd.ctr.as<uint32_t>();
	g.fl = pd.flags_arg;
	g.err = pd.err_dev;
	g.timeout_ticks = pd.timeout_ticks;
	g.poll = poll ? 1 : 0;
	g.nranks = (uint32_t)pd.nranks;
	g.rank = (uint32_t)pd.rank;
	g.per = pd.per;
	const uint64_t pad = pd.per * (uint64_t)pd.nranks;
	const int kb = what == 1 ? PB_W16 : PB_STATE;
	for (int p = 0; p < pd.nranks; ++p) g.peer[p] = (const uint8_t*)pd.host_ptr[(size_t)kb * pd.nranks + p];
	if (what == 1) {
		g.local[0] = (uint8_t*)w16.p;
		g.elem_bytes[0] = 2;
	} else {
		void* loc[4] = {w32.p, m1.p, m2.p, steps.p};
		for (int k = 0; k < 4; ++k) {
			g.local[k] = (uint8_t*)loc[k];
			g.peer_offset[k] = (uint64_t)k * pad * 4;
			g.elem_bytes[k] = 4;
		}
	}
	uint32_t maxb = 0;
	for (int k = 0; k < what; ++k) maxb = std::max(maxb, g.elem_bytes[k]);
	const uint64_t units = pd.per * maxb / 16;  // 16-byte units of one rank's shard
	const uint32_t cap = poll ? (pd.shared_device ? 1u : 64u) : 1024u;
	const uint32_t nx = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(div_round_up(units, 256), cap));
	hipLaunchKernelGGL(k_peer_gather, dim3(nx, pd.nranks, what), dim3(256), 0, st, g);
	TCNN_HIP_CHECK(hipGetLastError());
}

void TrainerHost::dp_peer_gather_state(hipStream_t st) {
	PeerDp& pd = *peer;
	pd.check();
	const uint64_t lo = std::min<uint64_t>(n_params, (uint64_t)pd.rank * pd.per), hi = std::min<uint64_t>(n_params, lo + pd.per);
	if (hi > lo)
		hipLaunchKernelGGL(k_peer_stage, dim3(div_round_up(hi - lo, 256)), dim3(256), 0, st, w32.as<float>(), m1.as<float>(), m2.as<float>(),
		                   steps.as<uint32_t>(), (uint32_t*)pd.x[PB_STATE], lo, hi - lo, pd.per * (uint64_t)pd.nranks, pd.ctr.as<uint32_t>());
	TCNN_HIP_CHECK(hipGetLastError());
	peer_wait(st, CTR_SYNC, SLOT_GATHER, 1);
	peer_gather(st, 4, false);
	TCNN_HIP_CHECK(hipStreamSynchronize(st));
	pd.check();
	dp_state_partial = false;
}

// collective: completes the sharded state, then waits until every rank has stopped reading this
// rank's mirrors before the mappings are closed and the mirrors freed
void TrainerHost::dp_peer_detach() {
	if (!peer) return;
	if (peer->attached) {
		if (dp_state_partial) dp_peer_gather_state(nullptr);
		peer_wait(nullptr, CTR_SYNC, SLOT_DETACH, 1);
		TCNN_HIP_CHECK(hipDeviceSynchronize());
	}
	peer.reset();
	peer_attached = false;
	peer_nranks = 1;
	dp_sharded = false;
	dp_state_partial = false;
	grad_scale = grad_scale_user;
	if (graph) set_graph(use_graph);
}

void TrainerHost::dp_peer_abandon() {
	if (!peer) return;
	TCNN_HIP_CHECK(hipDeviceSynchronize());
	peer.reset();
	peer_attached = false;
	peer_nranks = 1;
	dp_sharded = false;
	dp_state_partial = false;
	grad_scale = grad_scale_user;
}

}  // namespace tcnn_amd
