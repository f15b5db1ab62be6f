"""Data-parallel training over torch.distributed (RCCL over xGMI on MI355X, gloo on CPU).

The hot path shards by batch: each rank runs the training step on its own points
with run_optimizer=False, the fp32 gradient sums ([network | grid], the buffer Adam reads) are summed
across ranks, and every rank applies the same Adam step with gradient scale 1/N. Each shard's loss
normalises by its own B_r*dims (reference relative_l2.h:64, l2.h:64), so (1/N) * sum_r grad_r is the
gradient of the mean loss over all N*B_r points. Adam's "skip grid entries whose gradient is zero"
(reference adam.h:76-79) therefore sees the reduced gradient on every rank and the replicas stay
identical.

Exchange schedule (network parameters first, as the reference orders its parameter buffer,
network_with_input_encoding.h:115-122): the step runs in two parts; the all-reduce of the network
gradients (28 KB for config_hash) is issued asynchronously after part 0 and runs on the
communicator's stream while part 1 -- the grid backward -- runs on the compute stream; the grid
gradients (2.8 MB) follow. Both are waited for on the compute stream (no host synchronisation)
before Adam.

allreduce_dtype="fp16" halves the exchange: every rank pre-divides its gradient by N and rounds it
to fp16 (the reference's gradient buffer is __half, trainer.h:327), the fp16 sum is taken by the
collective, and Adam reads it with scale 1. The default fp32 exchange keeps the single-GPU
numerics (one fp16 rounding of the reduced sum).

exchange="peer": the exchange through the ranks' peer-mapped memory (PeerExchange, csrc/dp_peer.hip):
sharded, no collective library in the step, one C-ABI call per step. It is the default on GPU ranks
(exchange="auto": "peer" when the process group's backend is nccl/RCCL, else "torch", e.g. the gloo
rehearsal on CPU), with a collective fallback to "engine" when some rank cannot map its peers.
Teardown of a peer attachment is collective: call close() (or gather_state() and close()) on every
rank before the trainer goes away.

exchange="engine": the same exchange runs inside the engine instead (EngineComm, tcnn_trainer_set_dp):
one RCCL communicator created from a unique id broadcast over torch.distributed, the collectives
issued by the training step itself on its stream (network part overlapped with the grid backward),
so a data-parallel step is one C-ABI call that a hipGraph can capture. exchange="torch" drives
torch.distributed collectives from Python -- also the gloo rehearsal on CPU.

shard_optimizer=True (ZeRO-1 style): instead of the all-reduce,
the fp32 gradient sums are reduce-scattered (each rank receives the sum of one contiguous 1/N of the
parameter vector), each rank runs Adam on its shard only (Trainer.optimizer_step_range, grad scale
1/N), and the updated fp16 parameters -- what the next step's kernels read -- are all-gathered.
Per step that moves (N-1)/N of 4 + 2 bytes per parameter instead of 2 (N-1)/N of 4, and Adam, whose
cost does not shrink with the per-rank batch (36 B per parameter), runs on 1/N of the parameters.
The fp32 master weights and Adam state stay sharded (each rank's are current on its own shard);
gather_state() all-gathers the fp32 masters, both Adam moments and the per-parameter step counts,
and the trainer refuses serialize(optimizer=True) until it has run. For two ranks the result is
bit-identical to the all-reduce schedule (a + b is the same sum either way).

Batch sharding: strong scaling splits one global batch into contiguous shards (shard_bounds);
weak scaling gives every rank its own full batch. Both use the same step.
"""
import ctypes

import torch
import torch.distributed as dist


def allreduce_gradients(grad, group=None):
    """Sum `grad` (a torch tensor, fp32) across ranks in place; returns the 1/N scale Adam must apply."""
    world = dist.get_world_size(group)
    if world > 1:
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)
    return 1.0 / world


def shard_bounds(n, rank, world):
    """Contiguous shard [lo, hi) of n points for rank (strong scaling)."""
    per = n // world
    return rank * per, (rank + 1) * per if rank < world - 1 else n


def shard(x, rank, world):
    """Rank's contiguous shard of a [n, ...] tensor (strong scaling)."""
    lo, hi = shard_bounds(x.shape[0], rank, world)
    return x[lo:hi]


class EngineComm:
    """An engine data-parallel communicator (tcnn_dp_comm_create, RCCL over xGMI) for the ranks of
    `group`: rank 0 draws the unique id, torch.distributed broadcasts it (any backend), every rank
    creates its communicator on its current device."""

    def __init__(self, group=None):
        from tinycudann import _lib as L
        self._L = L
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        uid = torch.zeros(128, dtype=torch.uint8)
        if self.rank == 0:
            L.check(L.lib().tcnn_dp_unique_id(ctypes.c_void_p(uid.data_ptr())))
        on_gpu = dist.get_backend(group) == "nccl"
        t = uid.cuda() if on_gpu else uid
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        uid = t.cpu().contiguous()
        self.h = L.check_ptr(L.lib().tcnn_dp_comm_create(ctypes.c_void_p(uid.data_ptr()), self.world, self.rank))

    def __del__(self):
        try:
            self._L.lib().tcnn_dp_comm_destroy(self.h)
        except Exception:
            pass


class PeerExchange:
    """The engine's exchange over peer-mapped device memory (tcnn_trainer_dp_peer_*, csrc/dp_peer.hip):
    every rank exports IPC handles of its buffers, the blobs are all-gathered over torch.distributed
    (any backend, once), every rank attaches them. From then on the trainer's training_step exchanges
    through the peers' memory by itself: sharded Adam on the sum of the ranks' gradients read over
    xGMI, then a gather of the other shards' fp16 parameters -- no collective launch per step."""

    def __init__(self, trainer, group=None, timeout_s=None):
        from tinycudann import _lib as L
        self._L = L
        self.trainer = trainer
        self.attached = False
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if timeout_s is not None:  # default: TCNN_PEER_TIMEOUT_S or 300 s
            L.check(L.lib().tcnn_trainer_dp_peer_set_timeout(trainer.h, float(timeout_s)))
        n = int(L.lib().tcnn_dp_peer_blob_bytes())
        blob = (ctypes.c_uint8 * n)()
        ok = L.lib().tcnn_trainer_dp_peer_export(trainer.h, self.world, self.rank, ctypes.byref(blob)) == 0
        err = "" if ok else L.lib().tcnn_last_error().decode()
        blobs = [None] * self.world
        dist.all_gather_object(blobs, bytes(blob) if ok else None, group=group)
        if ok and all(b is not None for b in blobs):
            allb = (ctypes.c_uint8 * (n * self.world)).from_buffer_copy(b"".join(blobs))
            ok = L.lib().tcnn_trainer_dp_peer_attach(trainer.h, ctypes.byref(allb)) == 0
            if not ok:
                err = L.lib().tcnn_last_error().decode()
        else:
            ok = False
        # collective verdict: either every rank attached, or none keeps its attachment
        oks = [None] * self.world
        dist.all_gather_object(oks, (ok, err), group=group)
        if not all(o[0] for o in oks):
            L.lib().tcnn_trainer_dp_peer_abandon(trainer.h)
            raise RuntimeError("peer exchange unavailable: " + "; ".join(f"rank {r}: {o[1]}" for r, o in enumerate(oks) if not o[0]))
        trainer._dp_state_partial = False
        self.attached = True

    def detach(self):
        """collective: completes the sharded optimizer state, then closes the peer mappings (every
        rank calls it; idempotent)"""
        if self.attached:
            self.attached = False
            self._L.check(self._L.lib().tcnn_trainer_dp_peer_detach(self.trainer.h))

    close = detach

    def __del__(self):
        # no collective from a finaliser: a rank collected on its own (or while unwinding an exception)
        # would wait for peers that never match it. Only warn; the trainer's own destructor drops the
        # local mappings. close() -- or `with DataParallelTrainer(...)` -- is the teardown path.
        if getattr(self, "attached", False):
            import warnings
            warnings.warn("PeerExchange collected while attached: call close() on every rank (collective) "
                          "before the trainer goes away; the sharded optimizer state was not gathered",
                          ResourceWarning, stacklevel=2)


class DataParallelTrainer:
    """Wraps tinycudann.Trainer: training_step = local fwd/bwd, all-reduce (overlapped), Adam."""

    def __init__(self, trainer, group=None, overlap=True, allreduce_dtype="fp32", shard_optimizer=False, exchange="auto",
                 peer_fallback=True, peer_timeout_s=None):
        assert allreduce_dtype in ("fp32", "fp16")
        assert exchange in ("auto", "torch", "engine", "peer")
        if exchange == "auto":  # the peer exchange on GPU ranks (RCCL process group), torch.distributed otherwise
            gpu = dist.is_initialized() and dist.get_backend(group) == "nccl"
            exchange = "peer" if gpu and allreduce_dtype == "fp32" else "torch"
        assert not (shard_optimizer and allreduce_dtype == "fp16"), "the sharded optimizer exchanges fp32 gradient sums"
        assert not (exchange in ("engine", "peer") and allreduce_dtype == "fp16"), "the engine exchanges sum fp32 gradients"
        self.trainer = trainer
        self.group = group
        self.overlap = overlap
        self.dtype = allreduce_dtype
        self.shard_optimizer = shard_optimizer
        self.exchange = exchange
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.comm = None
        if self.world > 1 and exchange == "peer":
            self.shard_optimizer = True  # the peer exchange is the sharded schedule
            try:
                self.comm = PeerExchange(trainer, group, timeout_s=peer_timeout_s)
            except RuntimeError as e:
                if not peer_fallback:
                    raise
                # every rank raised together (collective verdict): take the engine's RCCL exchange instead
                import warnings
                warnings.warn(f"{e}; falling back to the engine's RCCL exchange (sharded)")
                self.exchange = exchange = "engine"
        if self.world > 1 and exchange == "engine":
            self.comm = EngineComm(group)
            trainer.set_dp(self.comm, sharded=self.shard_optimizer)
        elif self.world > 1 and exchange == "peer":
            pass  # attached above; the engine scales the gradient by 1/N itself
        elif self.world > 1 and shard_optimizer:
            self.rank = dist.get_rank(group)
            n = trainer.n_params
            self._per = (n + self.world - 1) // self.world
            padded = self._per * self.world
            self._lo = min(n, self.rank * self._per)
            self._hi = min(n, self._lo + self._per)
            self._grad = trainer.gradients_fp32()
            self._w16 = trainer.params()
            self._gpad = torch.zeros(padded, dtype=torch.float32, device=self._grad.device)
            self._gshard = torch.empty(self._per, dtype=torch.float32, device=self._grad.device)
            self._wpad = torch.zeros(padded, dtype=torch.float16, device=self._grad.device)
            self._wshard = torch.zeros(self._per, dtype=torch.float16, device=self._grad.device)
            trainer.set_gradient_scale(1.0 / self.world)
        elif self.world > 1:
            self._grad = trainer.gradients_fp32()
            nm = trainer.n_network_params
            self._views = (self._grad[:nm], self._grad[nm:])
            if self.dtype == "fp16":
                self._h = torch.empty(self._grad.numel(), dtype=torch.float16, device=self._grad.device)
                self._hviews = (self._h[:nm], self._h[nm:])
                trainer.set_gradient_scale(1.0)
            else:
                trainer.set_gradient_scale(1.0 / self.world)

    def _reduce_async(self, k):
        if self.dtype == "fp16":
            torch.mul(self._views[k], 1.0 / self.world, out=self._views[k])
            self._hviews[k].copy_(self._views[k])
            return dist.all_reduce(self._hviews[k], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        return dist.all_reduce(self._views[k], op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def _sharded_step(self, input, target):
        t, n = self.trainer, self.trainer.n_params
        t.training_step(input, target, run_optimizer=False)
        self._gpad[:n].copy_(self._grad)
        dist.reduce_scatter_tensor(self._gshard, self._gpad, op=dist.ReduceOp.SUM, group=self.group)
        if self._hi > self._lo:
            self._grad[self._lo:self._hi].copy_(self._gshard[:self._hi - self._lo])
        t.optimizer_step_range(self._lo, self._hi)
        if self._hi > self._lo:
            self._wshard[:self._hi - self._lo].copy_(self._w16[self._lo:self._hi])
        dist.all_gather_into_tensor(self._wpad, self._wshard, group=self.group)
        self._w16.copy_(self._wpad[:n])
        self.trainer._dp_state_partial = True

    def _gather(self, v):
        """all-gather this rank's shard [lo, hi) of the trainer buffer view v into every rank's v"""
        n = self.trainer.n_params
        buf = torch.zeros(self._per * self.world, dtype=v.dtype, device=v.device)
        mine = torch.zeros(self._per, dtype=v.dtype, device=v.device)
        if self._hi > self._lo:
            mine[:self._hi - self._lo].copy_(v[self._lo:self._hi])
        dist.all_gather_into_tensor(buf, mine, group=self.group)
        v.copy_(buf[:n])

    def gather_state(self):
        """All-gather the sharded optimizer state -- fp32 master weights, both Adam moments and the
        per-parameter step counts -- so every rank holds the full vectors, e.g. before
        serialize(optimizer=True) (which refuses to run until then)."""
        if self.world == 1 or not self.shard_optimizer:
            return
        if self.exchange in ("engine", "peer"):
            self.trainer.dp_gather_state()
            return
        m1, m2, steps = self.trainer.optimizer_state()
        for v in (self.trainer.params_fp32(), m1, m2, steps):
            self._gather(v)
        self.trainer._dp_state_partial = False

    gather_master = gather_state  # the round-2 name (it gathered only the masters)

    def close(self):
        """collective teardown: detaches the peer exchange (completing the sharded optimizer state) or
        the engine communicator; every rank calls it before its trainer goes away"""
        if isinstance(self.comm, PeerExchange):
            self.comm.close()
        elif isinstance(self.comm, EngineComm):
            self.trainer.set_dp(None)
        self.comm = None

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        # on an exception the ranks may not all reach this point: skip the collective teardown then
        # (PeerExchange.__del__ warns) rather than wait on peers that never arrive
        if exc_type is None:
            self.close()
        return False

    def training_step(self, input, target):
        if self.world == 1 or self.exchange in ("engine", "peer"):
            self.trainer.training_step(input, target, run_optimizer=True)
            return
        if self.shard_optimizer:
            self._sharded_step(input, target)
            return
        if self.overlap:
            self.trainer.training_step_part(input, target, 0)
            w_net = self._reduce_async(0)  # network gradients travel while the grid backward runs
            self.trainer.training_step_part(input, target, 1)
            w_grid = self._reduce_async(1)
            w_net.wait()
            w_grid.wait()
        else:
            self.trainer.training_step(input, target, run_optimizer=False)
            self._reduce_async(0).wait()
            self._reduce_async(1).wait()
        if self.dtype == "fp16":
            self._grad.copy_(self._h)
        self.trainer.optimizer_step()
