"""Host-time breakdown of the torch training step -- the NeuralBTF caller's path, reference
samples/mlp_learning_an_image_pytorch.py:159-170: tinycudann.NetworkWithInputEncoding forward, a
relative L2 in torch, loss.backward(), torch.optim.Adam -- on config_hash.json.

Per phase (forward / loss / zero_grad / backward / optimizer) the host time to issue it, averaged over
K steady-state steps with no synchronisation inside the loop, next to the GPU time per step (events)
and the Trainer's step (one C-ABI call). A step whose host time exceeds its GPU time is host-bound.
Also the number of GPU kernels one torch step launches (torch.profiler) by phase owner.

  python tools/torch_step_profile.py [--out profiles/r04_torch_step.json]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]


def run(iters, batches, fused_adam=False):
    import torch
    from bench import rgb_field_torch
    import tinycudann as tcnn
    from tinycudann import Trainer

    cfg = json.load(open(os.path.join(REPO, "tests", "golden", "config_hash.json")))
    rows = []
    for lb in batches:
        B = 1 << lb
        pos = torch.rand(B, 2, device="cuda")
        tgt = rgb_field_torch(pos)
        model = tcnn.NetworkWithInputEncoding(2, 3, cfg["encoding"], cfg["network"]).cuda()
        opt = torch.optim.Adam(model.parameters(), lr=0.01, fused=True) if fused_adam else torch.optim.Adam(model.parameters(), lr=0.01)
        phases = ["forward", "loss", "zero_grad", "backward", "optimizer"]
        host = dict.fromkeys(phases, 0.0)

        def step(record):
            t0 = time.perf_counter()
            out = model(pos)
            t1 = time.perf_counter()
            loss = ((out - tgt.to(out.dtype)) ** 2 / (out.detach() ** 2 + 0.01)).mean()
            t2 = time.perf_counter()
            opt.zero_grad()
            t3 = time.perf_counter()
            loss.backward()
            t4 = time.perf_counter()
            opt.step()
            t5 = time.perf_counter()
            if record:
                for k, (a, b) in zip(phases, ((t0, t1), (t1, t2), (t2, t3), (t3, t4), (t4, t5))):
                    host[k] += b - a

        for _ in range(20):
            step(False)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        h0 = time.perf_counter()
        for _ in range(iters):
            step(True)
        h1 = time.perf_counter()
        ev[1].record()
        torch.cuda.synchronize()
        wall = ev[0].elapsed_time(ev[1]) * 1e-3 / iters
        # GPU busy time of one step: the same step issued while the GPU is kept waiting on a long
        # kernel first, so issue overhead is hidden and the events bracket only GPU execution
        busy = None
        try:
            torch.cuda._sleep(int(2e8))
            e2 = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            torch.cuda.synchronize()
            torch.cuda._sleep(int(5e8))
            e2[0].record()
            for _ in range(10):
                step(False)
            e2[1].record()
            torch.cuda.synchronize()
            busy = e2[0].elapsed_time(e2[1]) * 1e-3 / 10
        except Exception:
            pass
        # kernel count per step
        n_kernels = None
        try:
            from torch.profiler import ProfilerActivity, profile
            with profile(activities=[ProfilerActivity.CUDA]) as prof:
                step(False)
                torch.cuda.synchronize()
            n_kernels = sum(1 for e in prof.events() if e.device_type.name == "CUDA")
        except Exception:
            pass
        t = Trainer(2, 3, cfg, seed=1337)
        for _ in range(20):
            t.training_step(pos, tgt)
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(iters):
            t.training_step(pos, tgt)
        ev[1].record()
        torch.cuda.synchronize()
        tr = ev[0].elapsed_time(ev[1]) * 1e-3 / iters
        row = {"batch": B, "optimizer": "torch.optim.Adam(fused=True)" if fused_adam else "torch.optim.Adam (default)",
               "torch_step_s": wall, "torch_host_issue_s": (h1 - h0) / iters, "torch_gpu_busy_s": busy,
               "host_s_by_phase": {k: v / iters for k, v in host.items()}, "gpu_kernels_per_step": n_kernels,
               "trainer_step_s": tr, "torch_over_trainer": wall / tr}
        rows.append(row)
        print(json.dumps(row), flush=True)
        del model, opt, t
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--batches", default="16,18", help="log2 batch sizes, comma separated")
    args = ap.parse_args()
    res = {"what": "torch NetworkWithInputEncoding training step (reference mlp_learning_an_image_pytorch.py:159-170): "
                   "host issue time per phase, GPU time per step, vs Trainer::training_step; config_hash.json",
           "rows": run(args.iters, tuple(int(b) for b in args.batches.split(","))) +
                   run(args.iters, tuple(int(b) for b in args.batches.split(",")), fused_adam=True)}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
