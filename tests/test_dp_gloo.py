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


class _FakeTrainer:
    """Stands in for tinycudann.Trainer on the CPU: deterministic per-rank gradients, records what
    the optimizer step would read (gradient buffer x gradient scale)."""

    def __init__(self, rank, n_net=8, n=40):
        self.rank = rank
        self.n_network_params = n_net
        self.g = torch.zeros(n, dtype=torch.float32)
        self.scale = 1.0
        self.parts = []
        self.seen = None

    def gradients_fp32(self):
        return self.g

    def set_gradient_scale(self, s):
        self.scale = s

    def _fill(self, lo, hi):
        idx = torch.arange(lo, hi, dtype=torch.float32)
        self.g[lo:hi] = (idx + 1.0) * (self.rank + 1) * 0.37

    def training_step_part(self, x, t, part):
        self.parts.append(part)
        if part == 0:
            self._fill(0, self.n_network_params)
        else:
            self._fill(self.n_network_params, self.g.numel())

    def training_step(self, x, t, run_optimizer=True):
        assert not run_optimizer
        self._fill(0, self.g.numel())

    def optimizer_step(self):
        self.seen = (self.g * self.scale).clone()


class _FakeShardTrainer(_FakeTrainer):
    """Adds what the sharded optimizer uses: fp16 parameter view, fp32 masters and a ranged Adam
    that writes the gradient it reads (x grad scale) into both."""

    def __init__(self, rank, n_net=8, n=41):
        super().__init__(rank, n_net, n)
        self.n_params = n
        self.w16 = torch.zeros(n, dtype=torch.float16)
        self.w32 = torch.zeros(n, dtype=torch.float32)
        self.m1 = torch.zeros(n, dtype=torch.float32)
        self.m2 = torch.zeros(n, dtype=torch.float32)
        self.steps = torch.zeros(n, dtype=torch.int32)
        self.ranges = []

    def params(self):
        return self.w16

    def params_fp32(self):
        return self.w32

    def optimizer_state(self):
        return self.m1, self.m2, self.steps

    def optimizer_step_range(self, lo, hi):
        self.ranges.append((lo, hi))
        self.w32[lo:hi] = self.g[lo:hi] * self.scale
        self.w16[lo:hi] = self.w32[lo:hi].half()
        self.m1[lo:hi] = self.w32[lo:hi] * 0.1
        self.m2[lo:hi] = self.w32[lo:hi] * 0.01
        self.steps[lo:hi] += 1


def _sched_worker(rank, world, port, out_q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [repo, os.path.join(repo, "neuralbtf-tiny-cuda-nn_amd"), here]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tinycudann.parallel import DataParallelTrainer, shard
    res = {}
    for overlap in (True, False):
        for dtype in ("fp32", "fp16"):
            t = _FakeTrainer(rank)
            dp = DataParallelTrainer(t, overlap=overlap, allreduce_dtype=dtype)
            dp.training_step(None, None)
            res[(overlap, dtype)] = (t.seen.numpy(), t.parts)
    t = _FakeShardTrainer(rank)
    dp = DataParallelTrainer(t, shard_optimizer=True)
    dp.training_step(None, None)
    w16 = t.w16.clone()
    partial = t._dp_state_partial
    dp.gather_state()
    res["zero"] = (w16.float().numpy(), t.w32.numpy(), t.ranges, t.m1.numpy(), t.m2.numpy(), t.steps.numpy(), partial,
                   t._dp_state_partial)
    x = torch.arange(10 * 3).reshape(10, 3)
    res["shard"] = shard(x, rank, world).numpy()
    out_q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_exchange_schedule_and_sharding():
    """DataParallelTrainer on gloo world 2 (CPU): the overlapped two-part schedule (network
    gradients first) and the plain one give the same Adam input = mean of the rank gradients; the
    fp16 exchange = fp16 sum of the pre-divided fp16 gradients; strong-scaling shards tile the
    global batch."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sched_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    idx = np.arange(40, dtype=np.float32)
    mean = ((idx + 1) * 1 * np.float32(0.37) + (idx + 1) * 2 * np.float32(0.37)) / 2
    for r in range(world):
        g_over, parts = res[r][(True, "fp32")]
        assert parts == [0, 1]
        np.testing.assert_allclose(g_over, mean, rtol=1e-6)
        np.testing.assert_array_equal(g_over, res[r][(False, "fp32")][0])
        g16 = res[r][(True, "fp16")][0]
        h = [((idx + 1) * (k + 1) * np.float32(0.37) / 2).astype(np.float16) for k in range(world)]
        np.testing.assert_array_equal(g16, (h[0] + h[1]).astype(np.float32))
    np.testing.assert_array_equal(np.concatenate([res[0]["shard"], res[1]["shard"]]), np.arange(30).reshape(10, 3))
    # sharded optimizer over 41 parameters (padded to 42): rank 0 updates [0, 21), rank 1 [21, 41);
    # afterwards every rank holds the whole fp16 vector and, after gather_state, the fp32 one and the Adam state
    idx41 = np.arange(41, dtype=np.float32)
    mean41 = ((idx41 + 1) * np.float32(0.37) + (idx41 + 1) * 2 * np.float32(0.37)) / 2
    for r in range(world):
        w16, w32, ranges, m1, m2, steps, partial, partial_after = res[r]["zero"]
        assert ranges == [(0, 21)] if r == 0 else ranges == [(21, 41)]
        np.testing.assert_allclose(w32, mean41, rtol=1e-6)
        np.testing.assert_array_equal(w16, w32.astype(np.float16).astype(np.float32))
        # gather_state: the Adam moments and step counts of every shard reach every rank, and the
        # serialize(optimizer=True) guard is lifted
        np.testing.assert_array_equal(m1, w32 * np.float32(0.1))
        np.testing.assert_array_equal(m2, w32 * np.float32(0.01))
        np.testing.assert_array_equal(steps, np.ones(41, np.int32))
        assert partial and not partial_after


class _FakePeerLib:
    """The peer-exchange C-ABI as PeerExchange calls it, with scripted failures per rank."""

    def __init__(self, rank, fail_export=(), fail_attach=()):
        self.rank, self.fail_export, self.fail_attach = rank, fail_export, fail_attach
        self.calls = []
        self.err = b""

    def tcnn_dp_peer_blob_bytes(self):
        return 16

    def tcnn_trainer_dp_peer_export(self, h, world, rank, blob):
        self.calls.append("export")
        if rank in self.fail_export:
            self.err = b"hipIpcGetMemHandle failed (scripted)"
            return 1
        return 0

    def tcnn_trainer_dp_peer_attach(self, h, blobs):
        self.calls.append("attach")
        if self.rank in self.fail_attach:
            self.err = b"hipIpcOpenMemHandle failed (scripted)"
            return 1
        return 0

    def tcnn_trainer_dp_peer_abandon(self, h):
        self.calls.append("abandon")
        return 0

    def tcnn_last_error(self):
        return self.err


def _peer_verdict_worker(rank, world, port, out_q):
    import sys
    import types
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [repo, os.path.join(repo, "neuralbtf-tiny-cuda-nn_amd"), here]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tinycudann import _lib as L
    from tinycudann.parallel import PeerExchange
    res = {}
    for case, kw in (("ok", {}), ("export", {"fail_export": (1,)}), ("attach", {"fail_attach": (0,)})):
        fake = _FakePeerLib(rank, **kw)
        L.lib = lambda fake=fake: fake
        t = types.SimpleNamespace(h=None, _dp_state_partial=True)
        try:
            PeerExchange(t)
            res[case] = ("attached", fake.calls, t._dp_state_partial)
        except RuntimeError as e:
            res[case] = (str(e), fake.calls, t._dp_state_partial)
    out_q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_peer_exchange_collective_verdict():
    """PeerExchange (tinycudann/parallel.py) attaches on every rank or on none: an export failure on
    rank 1, or an attach failure on rank 0, makes BOTH ranks raise (naming the failing rank) and drop
    what they had (abandon), so DataParallelTrainer(peer_fallback=True) falls back on every rank
    together; the C-ABI is scripted (CPU, gloo world 2)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_peer_verdict_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        msg, calls, partial = res[r]["ok"]
        assert msg == "attached" and calls == ["export", "attach"] and partial is False
        msg, calls, _ = res[r]["export"]
        assert "rank 1" in msg and "hipIpcGetMemHandle" in msg
        assert calls[-1] == "abandon" and "attach" not in calls  # nobody attaches when an export failed
        msg, calls, _ = res[r]["attach"]
        assert "rank 0" in msg and "hipIpcOpenMemHandle" in msg and calls[-1] == "abandon"
