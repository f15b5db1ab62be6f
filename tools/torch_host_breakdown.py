"""Host-time breakdown of the torch Module path's own share:
per step at B = 2^16 on config_hash, the host time spent in Module.forward, in its C-ABI forward call,
in the autograd backward node (_module_function.backward), and in its C-ABI backward call -- wrapped
timers around the real functions, steady state, no synchronisation inside the loop.

  python tools/torch_host_breakdown.py [--out profiles/r05_torch_host.json]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--log2b", type=int, default=16)
    args = ap.parse_args()
    import torch
    from bench import rgb_field_torch
    import tinycudann as tcnn
    from tinycudann import _lib as L
    from tinycudann import modules as M

    cfg = json.load(open(os.path.join(REPO, "tests", "golden", "config_hash.json")))
    B = 1 << args.log2b
    pos = torch.rand(B, 2, device="cuda")
    tgt = rgb_field_torch(pos)
    model = tcnn.NetworkWithInputEncoding(2, 3, cfg["encoding"], cfg["network"]).cuda()
    opt = torch.optim.Adam(model.parameters(), lr=0.01, fused=True)
    acc = {}

    def timed(name, f):
        def g(*a, **k):
            t0 = time.perf_counter()
            r = f(*a, **k)
            acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
            return r
        return g

    lib = L.lib()
    real_fwd, real_bwd = lib.tcnn_module_forward, lib.tcnn_module_backward_scaled

    class LibProxy:
        def __getattr__(self, n):
            if n == "tcnn_module_forward":
                return timed("C-ABI forward call", real_fwd)
            if n == "tcnn_module_backward_scaled":
                return timed("C-ABI backward call", real_bwd)
            return getattr(lib, n)

    proxy = LibProxy()
    M.L.lib = lambda: proxy
    M.Module.forward = timed("Module.forward (total)", M.Module.forward)
    M._module_function.backward = staticmethod(timed("autograd backward node (total)", M._module_function.backward))

    phases = {}

    def step():
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
        for k, d in (("forward", t1 - t0), ("loss", t2 - t1), ("zero_grad", t3 - t2), ("backward", t4 - t3), ("optimizer", t5 - t4)):
            phases[k] = phases.get(k, 0.0) + d

    for _ in range(30):
        step()
    torch.cuda.synchronize()
    acc.clear()
    phases.clear()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    h0 = time.perf_counter()
    for _ in range(args.iters):
        step()
    h1 = time.perf_counter()
    e[1].record()
    torch.cuda.synchronize()
    n = args.iters
    res = {"batch": B, "step_us": e[0].elapsed_time(e[1]) * 1e3 / n, "host_issue_us": (h1 - h0) * 1e6 / n,
           "host_us_by_phase": {k: v * 1e6 / n for k, v in phases.items()},
           "host_us_inside": {k: v * 1e6 / n for k, v in acc.items()}}
    t = tcnn.Trainer(2, 3, cfg, seed=1337)
    for _ in range(20):
        t.training_step(pos, tgt)
    torch.cuda.synchronize()
    e[0].record()
    for _ in range(n):
        t.training_step(pos, tgt)
    e[1].record()
    torch.cuda.synchronize()
    res["trainer_step_us"] = e[0].elapsed_time(e[1]) * 1e3 / n
    res["torch_over_trainer"] = res["step_us"] / res["trainer_step_us"]
    print(json.dumps(res, indent=1))
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
