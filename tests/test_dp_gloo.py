"""World-size-2 data-parallel check on CPU (gloo): per-rank shard gradients (CPU oracle, the same
math the GPU kernels implement) summed by tinycudann.parallel.allreduce_gradients and scaled 1/N
equal the full-batch gradient, and one Adam step on the reduced gradient keeps replicas identical."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, out_q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [repo, os.path.join(repo, "neuralbtf-tiny-cuda-nn_amd"), here]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from helpers import CONFIG_HASH, make_batch
    from oracle import oracle as O
    from tinycudann.parallel import allreduce_gradients, shard_bounds
    pos, tgt = make_batch(B)
    lo, hi = shard_bounds(B, rank, world)
    om = O.OracleModel(CONFIG_HASH, 2, 3, seed=1337)
    om.train_step(pos[lo:hi], tgt[lo:hi], run_optimizer=False)
    g = torch.from_numpy(om.grad32.copy())
    scale = allreduce_gradients(g)
    g16 = O.f2h(g.numpy() * np.float32(scale))
    w32, w16 = om.w32.copy(), om.w16.copy()
    m1 = np.zeros_like(w32); m2 = np.zeros_like(w32); st = np.zeros(len(w32), np.uint32)
    O.adam_step(om.m.adam, om.n_mlp_params, 128.0, 1, w32, w16, g16, m1, m2, st)
    if rank == 0:
        out_q.put((g.numpy() * scale, w32))
    else:
        out_q.put(("w", w32))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_two_rank_gradient_allreduce_matches_full_batch():
    from helpers import CONFIG_HASH, make_batch, rel_err
    from oracle import oracle as O
    B, world = 2048, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g_avg = [r for r in res if not isinstance(r[0], str)][0][0]
    w_ranks = [r[1] for r in res]
    np.testing.assert_array_equal(w_ranks[0], w_ranks[1])  # replicas identical after Adam
    pos, tgt = make_batch(B)
    om = O.OracleModel(CONFIG_HASH, 2, 3, seed=1337)
    om.train_step(pos, tgt, run_optimizer=False)
    nm = om.n_mlp_params
    assert rel_err(g_avg[:nm], om.grad32[:nm]) < 2e-3
    assert rel_err(g_avg[nm:], om.grad32[nm:]) < 2e-3
