// dp.cpp -- data-parallel gradient exchange inside the engine: one RCCL
// communicator over the ranks of a batch-sharded job (one process per GPU, xGMI), driven from the
// trainer's step on the trainer's stream, so the whole data-parallel step is one C-ABI call that a
// hipGraph can capture. The reference has no multi-GPU path.
//
// RCCL is loaded on first use (dlopen of librccl.so.1 -- the copy the process already has, e.g.
// torch's, or ROCm's): a single-GPU process never loads it, and the library has no link-time
// dependency on it.
#include <dlfcn.h>

#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

#include "runtime.h"

namespace tcnn_amd {

namespace {
struct RcclApi {
	decltype(&ncclGetUniqueId) get_unique_id = nullptr;
	decltype(&ncclCommInitRank) comm_init_rank = nullptr;
	decltype(&ncclCommDestroy) comm_destroy = nullptr;
	decltype(&ncclAllReduce) all_reduce = nullptr;
	decltype(&ncclReduceScatter) reduce_scatter = nullptr;
	decltype(&ncclAllGather) all_gather = nullptr;
	decltype(&ncclGetErrorString) error_string = nullptr;
};

const RcclApi& rccl() {
	static std::once_flag once;
	static RcclApi api;
	static std::string err;
	std::call_once(once, [] {
		void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
		if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
		if (!h) {
			err = std::string("RCCL not found (librccl.so.1): ") + dlerror();
			return;
		}
		auto sym = [&](const char* n) {
			void* p = dlsym(h, n);
			if (!p && err.empty()) err = std::string("RCCL symbol missing: ") + n;
			return p;
		};
		api.get_unique_id = (decltype(api.get_unique_id))sym("ncclGetUniqueId");
		api.comm_init_rank = (decltype(api.comm_init_rank))sym("ncclCommInitRank");
		api.comm_destroy = (decltype(api.comm_destroy))sym("ncclCommDestroy");
		api.all_reduce = (decltype(api.all_reduce))sym("ncclAllReduce");
		api.reduce_scatter = (decltype(api.reduce_scatter))sym("ncclReduceScatter");
		api.all_gather = (decltype(api.all_gather))sym("ncclAllGather");
		api.error_string = (decltype(api.error_string))sym("ncclGetErrorString");
	});
	TCNN_CHECK(err.empty(), err);
	return api;
}

void check(ncclResult_t r, const char* what) {
	if (r != ncclSuccess) throw std::runtime_error(std::string(what) + " failed: " + rccl().error_string(r));
}
}  // namespace

void dp_unique_id(void* id) {
	ncclUniqueId u;
	check(rccl().get_unique_id(&u), "ncclGetUniqueId");
	std::memcpy(id, &u, sizeof(u));
}

DpComm::DpComm(const void* id, int n, int r) : nranks(n), rank(r) {
	TCNN_CHECK(n >= 1 && r >= 0 && r < n, "dp communicator: rank outside [0, nranks)");
	ncclUniqueId u;
	std::memcpy(&u, id, sizeof(u));
	ncclComm_t c = nullptr;
	check(rccl().comm_init_rank(&c, n, u, r), "ncclCommInitRank");
	comm = c;
	TCNN_HIP_CHECK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
	for (auto& e : ev) TCNN_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
}

DpComm::~DpComm() {
	if (cs) (void)hipStreamSynchronize(cs);
	for (auto e : ev)
		if (e) (void)hipEventDestroy(e);
	if (cs) (void)hipStreamDestroy(cs);
	if (comm) (void)rccl().comm_destroy((ncclComm_t)comm);
}

void DpComm::all_reduce_f32(float* buf, size_t n, hipStream_t st) {
	if (n) check(rccl().all_reduce(buf, buf, n, ncclFloat32, ncclSum, (ncclComm_t)comm, st), "ncclAllReduce");
}

void DpComm::reduce_scatter_f32(float* buf, size_t per, hipStream_t st) {
	check(rccl().reduce_scatter(buf, buf + (size_t)rank * per, per, ncclFloat32, ncclSum, (ncclComm_t)comm, st), "ncclReduceScatter");
}

void DpComm::all_gather(void* buf, size_t per_elems, int elem_bytes, hipStream_t st) {
	const ncclDataType_t t = elem_bytes == 2 ? ncclFloat16 : ncclUint32;  // a gather moves bit patterns
	check(rccl().all_gather((const uint8_t*)buf + (size_t)rank * per_elems * elem_bytes, buf, per_elems, t, (ncclComm_t)comm, st),
	      "ncclAllGather");
}

// ------------------------------------------------------------------------------------------
// the trainer's data-parallel step
// ------------------------------------------------------------------------------------------
static void grow_preserve(DevBuf& b, size_t bytes, size_t valid) {
	if (b.bytes >= bytes) return;
	DevBuf n;
	n.reserve(bytes);
	TCNN_HIP_CHECK(hipMemset(n.p, 0, bytes));
	if (b.p && valid) TCNN_HIP_CHECK(hipMemcpy(n.p, b.p, valid, hipMemcpyDeviceToDevice));
	std::swap(b.p, n.p);
	std::swap(b.bytes, n.bytes);
}

void TrainerHost::set_dp(DpComm* c, bool sharded) {
	// Leaving a sharded schedule (detach, re-attach, or switch to replicated) first completes every
	// rank's fp32 masters, Adam moments and step counts over the OLD communicator -- otherwise the next
	// step's Adam would run on state that is stale outside this rank's shard and overwrite the gathered
	// fp16 weights of the other shards. This makes set_dp collective whenever state is partial: every
	// rank of the old communicator calls it (as every rank calls the sharded step).
	// any call while a peer exchange is attached (attach or detach) would reset its scale and shard
	// state under it: refused, detach the peer exchange first
	TCNN_CHECK(!peer_attached, "set_dp: the trainer is attached to a peer exchange (detach it first)");
	if (dp && dp_sharded && dp_state_partial) dp_gather_state(nullptr);
	TCNN_HIP_CHECK(hipDeviceSynchronize());
	dp = c;
	dp_sharded = c && sharded;
	dp_state_partial = false;
	// Adam reads the SUM over ranks: the caller's own scale (tcnn_trainer_set_gradient_scale) times 1/N
	grad_scale = grad_scale_user / (float)dp_nranks();
	if (graph) set_graph(use_graph);  // drop captured graphs (their keys do not hold the exchange)
	if (!dp_sharded) return;
	// shard s owns parameters [s per, (s + 1) per); every per-parameter buffer is padded to N per so
	// the in-place reduce-scatter / all-gather address whole shards
	const uint64_t N = (uint64_t)c->nranks;
	dp_per = (n_params + N - 1) / N;
	const size_t pad = (size_t)(dp_per * N);
	grow_preserve(w32, pad * 4, n_params * 4);
	grow_preserve(w16, pad * 2, n_params * 2);
	grow_preserve(g16, pad * 2, n_params * 2);
	grow_preserve(g32, pad * 4, n_params * 4);
	grow_preserve(m1, pad * 4, n_params * 4);
	grow_preserve(m2, pad * 4, n_params * 4);
	grow_preserve(steps, pad * 4, n_params * 4);
	ws.wimage_valid = false;
}

// One data-parallel training step: this rank's forward / backward, the gradient sum across ranks on
// the communicator's stream -- the network gradients (first in the parameter vector,
// network_with_input_encoding.h:115-122) while the grid backward still runs -- then Adam with
// gradient scale 1/N on every parameter (all-reduce) or on this rank's shard followed by an
// all-gather of the fp16 parameters (sharded). Each shard's loss normalises by its own B * dims
// (relative_l2.h:64), so (1/N) sum_r grad_r is the gradient of the mean loss; Adam's zero-gradient
// skip (adam.h:76-79) sees the summed gradient on every rank.
void TrainerHost::training_step_dp(hipStream_t st, uint32_t B, const float* input, const float* target) {
	DpComm& c = *dp;
	NetworkHost& m = *model;
	const size_t nm = (size_t)n_mlp;
	float* g = g32.as<float>();
	mark(st, 0);
	if (overlapped_ok()) {
		m.fused_kernel(st, ws, B, input, target, n_output_dims, loss_scale, w16.p, false);
		launch_column_sums(st, ws.wgrad_partial.as<float>(), ws.n_fused_blocks, (uint32_t)n_mlp, g);
		launch_sum(st, ws.loss_partial.as<float>(), ws.n_loss_partials, d_loss.as<float>());
		if (!dp_sharded) {  // the network part travels while the grid backward runs
			TCNN_HIP_CHECK(hipEventRecord(c.ev[0], st));
			TCNN_HIP_CHECK(hipStreamWaitEvent(c.cs, c.ev[0], 0));
			c.all_reduce_f32(g, nm, c.cs);
		}
		mark(st, 1);
		m.grid_backward(st, ws, B, input);
		m.grid->backward_acc(st, ws.gbw, B, ws.dLdenc.p, 0, 0, g + nm);
		m.grid->reduce_items(st, ws.gbw, g + nm);
	} else {
		m.fwd_bwd(st, ws, B, input, target, n_output_dims, loss_scale, w16.p, nullptr, nullptr, g);
		launch_sum(st, ws.loss_partial.as<float>(), ws.n_loss_partials, d_loss.as<float>());
		mark(st, 1);
	}
	mark(st, 2);
	TCNN_HIP_CHECK(hipEventRecord(c.ev[1], st));
	TCNN_HIP_CHECK(hipStreamWaitEvent(c.cs, c.ev[1], 0));
	if (dp_sharded) c.reduce_scatter_f32(g, (size_t)dp_per, c.cs);
	else if (overlapped_ok()) c.all_reduce_f32(g + nm, (size_t)(n_params - nm), c.cs);
	else c.all_reduce_f32(g, (size_t)n_params, c.cs);
	TCNN_HIP_CHECK(hipEventRecord(c.ev[2], c.cs));
	TCNN_HIP_CHECK(hipStreamWaitEvent(st, c.ev[2], 0));
	last_B = B;
	if (dp_sharded) {
		const uint64_t lo = std::min<uint64_t>(n_params, (uint64_t)c.rank * dp_per), hi = std::min<uint64_t>(n_params, lo + dp_per);
		optimizer_step_range(st, lo, hi);
		c.all_gather(w16.p, (size_t)dp_per, 2, st);
		dp_state_partial = true;
	} else {
		optimizer_step(st);
	}
	mark(st, 3);
}

// All-gather the sharded optimizer state so every rank holds the full vectors (fp32 masters, Adam
// moments, per-parameter step counts), e.g. before serialize(with_optimizer).
void TrainerHost::dp_gather_state(hipStream_t st) {
	if (peer_attached) {
		if (dp_state_partial) dp_peer_gather_state(st);
		return;
	}
	if (!dp || !dp_sharded || !dp_state_partial) return;
	for (DevBuf* b : {&w32, &m1, &m2, &steps}) dp->all_gather(b->p, (size_t)dp_per, 4, st);
	TCNN_HIP_CHECK(hipStreamSynchronize(st));
	dp_state_partial = false;
}

}  // namespace tcnn_amd
