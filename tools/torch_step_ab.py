"""The torch Module path's training step (the NeuralBTF caller's: tinycudann.NetworkWithInputEncoding,
RelativeL2 in torch, loss.backward(), torch.optim.Adam(fused=True)) with the C++ autograd node
(csrc/torch_ext.cpp, r06 default) and with the Python autograd.Function it replaces, in one process,
alternating; per step: GPU time (events over K steps), host issue time, host time by phase; and the
Trainer's step at the same batch for the ratio.

  python tools/torch_step_ab.py [--out profiles/r06_torch_host.json] [--log2b 16]
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
    from tinycudann import modules as M
    assert M._EXT is not None, "C++ autograd node not built"
    ext = M._EXT
    cfg = json.load(open(os.path.join(REPO, "tests", "golden", "config_hash.json")))
    B = 1 << args.log2b
    pos = torch.rand(B, 2, device="cuda")
    tgt = rgb_field_torch(pos)
    model = tcnn.NetworkWithInputEncoding(2, 3, cfg["encoding"], cfg["network"]).cuda()
    opt = torch.optim.Adam(model.parameters(), lr=0.01, fused=True)

    def run(use_ext):
        M._EXT = ext if use_ext else None
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
        return {"step_us": e[0].elapsed_time(e[1]) * 1e3 / n, "host_issue_us": (h1 - h0) * 1e6 / n,
                "host_us_by_phase": {k: round(v * 1e6 / n, 2) for k, v in phases.items()}}

    rows = {"cpp_node": [], "python_node": []}
    for _ in range(2):
        rows["cpp_node"].append(run(True))
        rows["python_node"].append(run(False))
    M._EXT = ext
    t = tcnn.Trainer(2, 3, cfg, seed=1337)
    for _ in range(20):
        t.training_step(pos, tgt)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(args.iters):
        t.training_step(pos, tgt)
    e[1].record()
    torch.cuda.synchronize()
    tr = e[0].elapsed_time(e[1]) * 1e3 / args.iters
    best = {k: min(v, key=lambda r: r["step_us"]) for k, v in rows.items()}
    res = {"what": __doc__.split("\n\n")[0], "batch": B, "runs": rows, "trainer_step_us": tr,
           "torch_over_trainer": {k: v["step_us"] / tr for k, v in best.items()}}
    print(json.dumps(res, indent=1))
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
