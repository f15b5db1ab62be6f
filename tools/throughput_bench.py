"""Throughput of the reference README's other published benchmarks (BASELINE.md rows 18-20,
reference README.md:8 + data/readme/fully-fused-vs-tensorflow.png, RTX 3090): FullyFusedMLP 64 and
128 neurons on data/config_oneblob.json (OneBlob 64 bins, RelativeL2, Adam), training and inference,
at batch 2^14 / 2^18 / 2^21, and the config_hash.json inference rate. Synthetic uniform inputs,
analytic targets, inputs resident in HBM; timing with torch.cuda events around K back-to-back calls
on one stream after W warm-up calls.

  python tools/throughput_bench.py [--out profiles/r02_throughput.json]
"""
import argparse
import copy
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]

PUBLISHED_3090 = {  # BASELINE.md rows 18-20 (samples/s)
    ("train", 64, 1 << 14): 1.2e8, ("train", 64, 1 << 18): 1.9e8, ("train", 64, 1 << 21): 1.98e8,
    ("train", 128, 1 << 14): 0.74e8, ("train", 128, 1 << 18): 0.93e8, ("train", 128, 1 << 21): 0.96e8,
    ("infer", 64, 1 << 18): 1.0e9, ("infer", 64, 1 << 21): 1.08e9, ("infer", 128, 1 << 18): 0.35e9, ("infer", 128, 1 << 21): 0.37e9,
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--graph", action="store_true", help="training steps replayed as hipGraphs")
    args = ap.parse_args()
    import torch
    from bench import rgb_field_torch
    from tinycudann import Trainer

    def timed(fn, iters, warm=5):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / iters * 1e-3

    base = json.load(open(os.path.join(REPO, "tests", "golden", "config_oneblob.json")))
    rows = []
    for W in (64, 128):
        cfg = copy.deepcopy(base)
        cfg["network"]["n_neurons"] = W
        t = Trainer(2, 3, cfg, seed=1337)
        if args.graph:
            t.set_graph(True)
        for lb in (14, 18, 21):
            B = 1 << lb
            pos = torch.rand(B, 2, device="cuda")
            tgt = rgb_field_torch(pos)
            it = max(5, args.iters if lb <= 18 else args.iters // 4)
            s = timed(lambda: t.training_step(pos, tgt), it)
            rows.append({"config": f"config_oneblob W{W} H{cfg['network']['n_hidden_layers']}", "mode": "train", "batch": B,
                         "engine": t.engine, "s_per_step": s, "samples_per_s": B / s, "steps_per_s": 1 / s,
                         "rtx3090_samples_per_s": PUBLISHED_3090.get(("train", W, B))})
            s = timed(lambda: t.inference(pos), it)
            rows.append({"config": f"config_oneblob W{W} H{cfg['network']['n_hidden_layers']}", "mode": "infer", "batch": B,
                         "engine": t.inference_engine, "s_per_call": s, "samples_per_s": B / s,
                         "rtx3090_samples_per_s": PUBLISHED_3090.get(("infer", W, B))})
            print(json.dumps(rows[-2]), flush=True)
            print(json.dumps(rows[-1]), flush=True)
        del t
    cfg = json.load(open(os.path.join(REPO, "tests", "golden", "config_hash.json")))
    cfg3 = copy.deepcopy(cfg)  # BASELINE configs[3]: HashGrid + W128/H4
    cfg3["network"]["n_neurons"], cfg3["network"]["n_hidden_layers"] = 128, 4
    for name, c in (("config_hash", cfg), ("configs3 HashGrid W128 H4", cfg3)):
        t = Trainer(2, 3, c, seed=1337)
        for lb in (18, 21):
            B = 1 << lb
            pos = torch.rand(B, 2, device="cuda")
            s = timed(lambda: t.inference(pos), args.iters)
            rows.append({"config": name, "mode": "infer", "batch": B, "engine": t.inference_engine, "s_per_call": s,
                         "samples_per_s": B / s})
            print(json.dumps(rows[-1]), flush=True)
        del t
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(0), "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
