"""The engine's data-parallel step (csrc/dp.cpp, tcnn_trainer_set_dp): RCCL collectives issued by the
training step itself. On a one-GPU box RCCL takes one rank per device ("Duplicate GPU detected"
otherwise), so these run a one-rank communicator: the step then goes through the whole exchange
code path -- part 0, the network all-reduce on the communicator's stream, part 1, the grid
all-reduce or the reduce-scatter / ranged Adam / all-gather of the sharded optimizer, the event
joins -- and must equal the plain single-GPU step bit for bit (sum over one rank, gradient scale 1).
Also under hipGraph capture, and the sharded state guard of serialize(optimizer=True). Multi-rank
schedules are covered by tests/test_dp_gloo.py (gloo, CPU) and the driver's 8-GPU run."""
import os
import socket

import numpy as np
import pytest

from helpers import CONFIG_HASH, make_batch, trainer_arrays

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def group():
    import torch
    import torch.distributed as dist
    assert torch.cuda.is_available()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    yield torch
    dist.destroy_process_group()


@pytest.mark.parametrize("sharded,graph", [(False, False), (True, False), (False, True), (True, True)])
def test_engine_dp_one_rank_equals_plain_step(group, sharded, graph):
    torch = group
    from tinycudann import Trainer
    from tinycudann.parallel import EngineComm
    comm = EngineComm()
    ref = Trainer(2, 3, CONFIG_HASH, seed=1337)
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    t.set_dp(comm, sharded=sharded)
    if graph:
        t.set_graph(True)
    B = 4096
    for s in range(5):
        pos, tgt = make_batch(B, step=s)
        p, g = torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda()
        ref.training_step(p, g)
        t.training_step(p, g)
        assert t.loss() == ref.loss(), s
    if sharded:
        with pytest.raises(Exception):
            t.serialize(optimizer=True)
        t.dp_gather_state()
    a, b = trainer_arrays(t), trainer_arrays(ref)
    for k in ("w16", "w32"):
        np.testing.assert_array_equal(a[k], b[k])
    for x, y in zip(t.optimizer_state(), ref.optimizer_state()):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())
    assert t.serialize(optimizer=True) == ref.serialize(optimizer=True)
    if graph:
        caps, reps = t.graph_stats()
        assert caps >= 1 and reps >= 1, (caps, reps)
    t.set_dp(None)


def test_detach_after_sharded_steps_keeps_state_and_scale(group):
    """Detaching a sharded trainer (set_dp(None)) with partial state completes the state first
    (csrc/dp.cpp set_dp), so local steps afterwards continue the same trajectory; the
    caller's gradient scale survives attach / detach (x 1/N only while attached)."""
    torch = group
    from tinycudann import Trainer
    from tinycudann.parallel import EngineComm
    comm = EngineComm()
    ref = Trainer(2, 3, CONFIG_HASH, seed=1337)
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    t.set_dp(comm, sharded=True)
    B = 4096
    for s in range(6):
        pos, tgt = make_batch(B, step=s)
        p, g = torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda()
        ref.training_step(p, g)
        if s == 3:
            t.set_dp(None)  # no explicit gather: set_dp must complete the sharded state itself
        t.training_step(p, g)
        assert t.loss() == ref.loss(), s
    assert t.serialize(optimizer=True) == ref.serialize(optimizer=True)
