"""The measured floor of the 8-way data-parallel step on one MI355X: the training
step of config_hash.json at B = 2^15 (one rank's shard of the 2^18 global batch at N = 8) without any
exchange, and the same step with each exchange schedule attached to a one-rank communicator (the
collectives run, over one rank). Reports per step: GPU time (events around K steps) and host issue
time (wall clock of issuing K steps, no synchronisation inside) -- a step is host-bound when the
second exceeds the first.

Schedules: plain (no exchange); peer (r04: the exchange through peer-mapped memory, csrc/dp_peer.hip,
on one rank); engine (tcnn_trainer_set_dp, RCCL issued by the step; replicated and
sharded, eager and hipGraph); torch (tinycudann.parallel.DataParallelTrainer's Python schedule over
torch.distributed/RCCL, replicated, overlapped; run with the wrapper's world size forced to 2 on a
one-rank group so its all-reduce path is taken -- the sums then run over one rank).

  python tools/dp_floor.py [--out profiles/r03_dp_floor.json]
"""
import argparse
import json
import os
import socket
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--batch-log2", type=int, default=15)
    ap.add_argument("--schedules", default="plain,engine,peer,torch", help="comma-separated subset")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from bench import rgb_field_torch
    from tinycudann import Trainer
    from tinycudann import parallel as P

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(s.getsockname()[1])
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    cfg = json.load(open(os.path.join(REPO, "tests", "golden", "config_hash.json")))
    B = 1 << args.batch_log2
    pos = torch.rand(B, 2, device="cuda")
    tgt = rgb_field_torch(pos)

    def measure(step):
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        host = (time.perf_counter() - t0) / args.steps
        b.record()
        torch.cuda.synchronize()
        gpu = a.elapsed_time(b) * 1e-3 / args.steps
        return {"gpu_us_per_step": gpu * 1e6, "host_issue_us_per_step": host * 1e6, "steps_per_s": 1.0 / gpu}

    rows = []

    def row(name, r):
        r = dict(r, schedule=name, batch=B)
        rows.append(r)
        print(json.dumps(r), flush=True)

    want = set(args.schedules.split(","))
    for graph in ((False, True) if "plain" in want else ()):
        t = Trainer(2, 3, cfg, seed=1337)
        t.set_graph(graph)
        row(f"plain{' graph' if graph else ''}", measure(lambda: t.training_step(pos, tgt)))
        del t
    comm = P.EngineComm() if "engine" in want else None
    for sharded in ((False, True) if "engine" in want else ()):
        for graph in (False, True):
            t = Trainer(2, 3, cfg, seed=1337)
            t.set_dp(comm, sharded=sharded)
            t.set_graph(graph)
            row(f"engine {'sharded' if sharded else 'replicated'}{' graph' if graph else ''}", measure(lambda: t.training_step(pos, tgt)))
            t.set_dp(None)
            del t
    # the peer-memory exchange (csrc/dp_peer.hip) on one rank: signal, wait, shard Adam over the
    # ranks' gradients, signal, wait, gather -- its whole per-step machinery, minus the link transfers
    if "peer" in want:
        t = Trainer(2, 3, cfg, seed=1337)
        px = P.PeerExchange(t)
        row("peer (xGMI exchange, sharded)", measure(lambda: t.training_step(pos, tgt)))
        px.detach()
        del t, px
    # loopback rehearsal of an N-rank peer step (debug_api.h tcnn_debug_peer_loopback): rank 0 of N whose
    # peers are all itself -- Adam on the 1/N shard over N mirrors, the gather of N - 1 shards, the polls
    # -- i.e. the per-rank kernels of the real N-rank step minus the link transfers
    for sch in sorted(w for w in want if w.startswith("peerloop")):
        n = int(sch[len("peerloop"):])
        t = Trainer(2, 3, cfg, seed=1337)
        from tinycudann import _lib as LL
        LL.check(LL.lib().tcnn_debug_peer_loopback(t.h, n))
        row(f"peer loopback N={n} (per-rank kernels of the {n}-rank step, no links)", measure(lambda: t.training_step(pos, tgt)))
        LL.check(LL.lib().tcnn_trainer_dp_peer_abandon(t.h))
        del t
    real_ws = P.dist.get_world_size
    P.dist.get_world_size = lambda group=None: 2  # take the wrapper's all-reduce path on the one-rank group
    try:
        if "torch" in want:
            t = Trainer(2, 3, cfg, seed=1337)
            dp = P.DataParallelTrainer(t, overlap=True)
            row("torch replicated overlapped (Python wrapper)", measure(lambda: dp.training_step(pos, tgt)))
            del dp, t
    finally:
        P.dist.get_world_size = real_ws
    dist.destroy_process_group()
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"what": __doc__.split("\n\n")[0], "device": torch.cuda.get_device_name(0), "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
