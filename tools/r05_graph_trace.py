"""Kernel-trace A/B of the eager and the hipGraph-replayed training step (config_hash, B = 2^15 and 2^18):
run under rocprofv3 --kernel-trace; prints per-step GPU time from events, and writes nothing else."""
import json, os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]
import torch
from bench import rgb_field_torch
from tinycudann import Trainer
cfg = json.load(open(os.path.join(REPO, "tests", "golden", "config_hash.json")))
for lb in (15, 18):
    B = 1 << lb
    pos = torch.rand(B, 2, device="cuda")
    tgt = rgb_field_torch(pos)
    for graph, user_stream in ((False, False), (True, False), (False, True), (True, True)):
        s = torch.cuda.Stream() if user_stream else torch.cuda.current_stream()
        with torch.cuda.stream(s):
            t = Trainer(2, 3, cfg, seed=1337)
            t.set_graph(graph)
            for _ in range(20):
                t.training_step(pos, tgt)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 200
            a.record()
            for _ in range(n):
                t.training_step(pos, tgt)
            b.record()
            torch.cuda.synchronize()
        print(json.dumps({"B": B, "graph": graph, "stream": "user" if user_stream else "null", "gpu_us_per_step": a.elapsed_time(b) * 1e3 / n,
                          "graph_stats": t.graph_stats()}), flush=True)
        del t
