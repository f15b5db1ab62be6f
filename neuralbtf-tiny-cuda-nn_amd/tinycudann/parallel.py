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

Batch sharding: strong scaling splits one global batch into contiguous shards (shard_bounds);
weak scaling gives every rank its own full batch. Both use the same step.
"""
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


class DataParallelTrainer:
    """Wraps tinycudann.Trainer: training_step = local fwd/bwd, all-reduce (overlapped), Adam."""

    def __init__(self, trainer, group=None, overlap=True, allreduce_dtype="fp32"):
        assert allreduce_dtype in ("fp32", "fp16")
        self.trainer = trainer
        self.group = group
        self.overlap = overlap
        self.dtype = allreduce_dtype
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if self.world > 1:
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

    def training_step(self, input, target):
        if self.world == 1:
            self.trainer.training_step(input, target, run_optimizer=True)
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
