"""Data-parallel path of the HIP engine with two ranks on one GPU (gloo all-reduce on device
tensors; the 8-GPU RCCL run is the driver's): shard gradients summed by
tinycudann.parallel.allreduce_gradients and scaled 1/N equal the single-process full-batch
gradient, and DataParallelTrainer keeps both replicas bit-identical under every
exchange schedule (overlapped, plain, pre-divided fp16, sharded optimizer)."""
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
    from tinycudann.parallel import DataParallelTrainer, allreduce_gradients, shard_bounds
    pos, tgt = make_batch(B)
    lo, hi = shard_bounds(B, rank, world)
    p, t = torch.from_numpy(pos[lo:hi]).cuda(), torch.from_numpy(tgt[lo:hi]).cuda()
    tr = Trainer(2, 3, CONFIG_HASH, seed=1337)
    tr.training_step(p, t, run_optimizer=False)
    g = tr.gradients_fp32().clone()
    scale = allreduce_gradients(g)
    g_avg = (g * scale).cpu().numpy()
    # full DataParallelTrainer steps on a fresh replica
    def run(gather=False, **kw):
        tr2 = Trainer(2, 3, CONFIG_HASH, seed=1337)
        dp = DataParallelTrainer(tr2, **kw)
        for s in range(3):
            pos_s, tgt_s = make_batch(B, step=s)
            dp.training_step(torch.from_numpy(pos_s[lo:hi]).cuda(), torch.from_numpy(tgt_s[lo:hi]).cuda())
        if gather:
            dp.gather_state()
        torch.cuda.synchronize()
        a = trainer_arrays(tr2)
        return a["w32"], a["w16"], bytes(tr2.serialize(optimizer=True))
    w_over, h_over, snap_over = run()         # two-part step, network all-reduce overlapping the grid backward
    w_plain = run(overlap=False)[0]           # whole backward, then the all-reduce
    w_half = run(allreduce_dtype="fp16")[0]   # pre-divided fp16 exchange
    w_shard, h_shard, snap_shard = run(gather=True, shard_optimizer=True)  # reduce-scatter, Adam on 1/N, all-gather
    q.put((rank, g_avg, w_over, w_plain, w_half, w_shard, h_shard, h_over, snap_over, snap_shard))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gpu_allreduce_matches_full_batch():
    import torch
    import torch.multiprocessing as mp
    from helpers import CONFIG_HASH, make_batch, rel_err, trainer_arrays
    B, world = 4096, 2
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
    np.testing.assert_array_equal(res[0][2], res[1][2])  # replicas identical
    np.testing.assert_array_equal(res[0][2], res[0][3])  # overlapped schedule == plain schedule, bit for bit
    np.testing.assert_array_equal(res[0][4], res[1][4])  # fp16 exchange: replicas identical too
    # close to the fp32 exchange: a gradient that rounds to 0 in one exchange and not the other is
    # skipped by Adam (adam.h:76-79) in one run only, so parameters differ by ~lr in a few places
    assert rel_err(res[0][4], res[0][2]) < 1e-2
    np.testing.assert_array_equal(res[0][1], res[1][1])
    # sharded optimizer (reduce-scatter, Adam on each rank's half, fp16 all-gather): bit-identical to
    # the all-reduce schedule for two ranks -- fp16 parameters, and the gathered fp32 masters
    for r in range(world):
        np.testing.assert_array_equal(res[r][6], res[r][7])
        np.testing.assert_array_equal(res[r][5], res[0][2])
        # the snapshot with optimizer state after gather_state (Adam moments and step counts of every
        # shard) is byte-identical to the replicated schedule's (a snapshot of a sharded
        # trainer must not carry partial moments)
        assert res[r][9] == res[r][8]
    from tinycudann import Trainer
    pos, tgt = make_batch(B)
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
    g_full = trainer_arrays(t)["g32"]
    nm = t.n_network_params
    assert rel_err(res[0][1][:nm], g_full[:nm]) < 2e-3
    assert rel_err(res[0][1][nm:], g_full[nm:]) < 2e-3
