"""The engine's peer-memory data-parallel exchange (csrc/dp_peer.hip, tinycudann.parallel.PeerExchange)
with two (and four) ranks on one GPU (IPC within a device): every rank exports IPC handles of its buffers, the
blobs are all-gathered over gloo, and each training_step sums the ranks' gradients for its shard
straight from the other rank's memory, runs Adam on the shard and copies the other shard's fp16
parameters. For two ranks the result must equal the replicated all-reduce schedule bit for bit
(g0 + g1 is one sum either way): fp32 masters, fp16 parameters and the optimizer snapshot after the
sharded state is gathered; the two replicas must be identical; detach is collective and leaves a
trainer that steps on alone."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [repo, os.path.join(repo, "neuralbtf-tiny-cuda-nn_amd"), here]
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from helpers import CONFIG_HASH, make_batch, trainer_arrays
    from tinycudann import Trainer
    from tinycudann.parallel import DataParallelTrainer, shard_bounds
    lo, hi = shard_bounds(B, rank, world)

    def run(**kw):
        tr = Trainer(2, 3, CONFIG_HASH, seed=1337)
        dp = DataParallelTrainer(tr, **kw)
        losses = []
        for s in range(4):
            pos_s, tgt_s = make_batch(B, step=s)
            dp.training_step(torch.from_numpy(pos_s[lo:hi]).cuda(), torch.from_numpy(tgt_s[lo:hi]).cuda())
            losses.append(tr.loss())
        dp.gather_state()
        torch.cuda.synchronize()
        a = trainer_arrays(tr)
        return tr, dp, a["w32"], a["w16"], bytes(tr.serialize(optimizer=True)), losses

    _, _, w_ref, h_ref, snap_ref, l_ref = run()  # replicated all-reduce (gloo), overlapped
    tr, dp, w_peer, h_peer, snap_peer, l_peer = run(exchange="peer")
    # detach (collective), then this rank trains on alone from the gathered state
    dp.comm.detach()
    pos_s, tgt_s = make_batch(B, step=9)
    tr.training_step(torch.from_numpy(pos_s[lo:hi]).cuda(), torch.from_numpy(tgt_s[lo:hi]).cuda())
    torch.cuda.synchronize()
    after = trainer_arrays(tr)["w32"]
    q.put((rank, w_ref, h_ref, snap_ref, l_ref, w_peer, h_peer, snap_peer, l_peer, bool(np.isfinite(after).all())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_peer_exchange_equals_allreduce(world):
    """2 ranks: bit-identical to the all-reduce. 4 ranks (1024 points each, padded shards of 178,888
    parameters): the peer sum runs in rank order g0+g1+g2+g3 while gloo's ring sums in its own order,
    so the comparison is within fp32 rounding; the replicas must still agree bit for bit."""
    import torch.multiprocessing as mp
    B = 4096
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        _, w_ref, h_ref, snap_ref, l_ref, w_peer, h_peer, snap_peer, l_peer, finite = r
        assert finite
        if world == 2:
            np.testing.assert_array_equal(w_peer, w_ref)
            np.testing.assert_array_equal(h_peer, h_ref)
            assert snap_peer == snap_ref
            assert l_peer == l_ref
        else:
            np.testing.assert_allclose(w_peer, w_ref, rtol=1e-3, atol=1e-6)
            np.testing.assert_allclose(np.asarray(l_peer), np.asarray(l_ref), rtol=1e-3)
    for r in res[1:]:  # the replicas agree
        np.testing.assert_array_equal(res[0][5], r[5])
        np.testing.assert_array_equal(res[0][6], r[6])
