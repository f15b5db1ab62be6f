"""Data-parallel training over torch.distributed (RCCL over xGMI on MI355X, gloo on CPU).

The hot path shards by batch: each rank runs Trainer::training_step on its own points (a weak-
scaling shard) with run_optimizer=False, the fp32 gradient sums ([network | grid], the buffer Adam
reads) are summed with ONE all-reduce, and every rank applies the same Adam step with gradient
scale 1/N. Each shard's RelativeL2 normalises by its own B_r*dims (reference relative_l2.h:64), so
(1/N) * sum_r grad_r is the gradient of the mean loss over all N*B_r points. Adam's "skip grid
entries whose gradient is zero" (reference adam.h:76-79) therefore sees the reduced gradient on
every rank and the replicas stay identical.
"""
import torch.distributed as dist


def allreduce_gradients(grad, group=None):
    """Sum `grad` (a torch tensor, fp32) across ranks in place; returns the 1/N scale Adam must apply."""
    world = dist.get_world_size(group)
    if world > 1:
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)
    return 1.0 / world


def shard_bounds(n, rank, world):
    """Contiguous shard [lo, hi) of n points for rank (strong-scaling helper)."""
    per = n // world
    return rank * per, (rank + 1) * per if rank < world - 1 else n


class DataParallelTrainer:
    """Wraps tinycudann.Trainer: training_step = local fwd/bwd, all-reduce, Adam."""

    def __init__(self, trainer, group=None):
        self.trainer = trainer
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self._grad = trainer.gradients_fp32() if self.world > 1 else None
        if self.world > 1:
            trainer.set_gradient_scale(1.0 / self.world)

    def training_step(self, input, target):
        if self.world == 1:
            self.trainer.training_step(input, target, run_optimizer=True)
            return
        self.trainer.training_step(input, target, run_optimizer=False)
        allreduce_gradients(self._grad, self.group)
        self.trainer.optimizer_step()
