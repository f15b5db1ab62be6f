"""configs[3] (HashGrid config_hash encoding + FullyFusedMLP W128/H4, B = 2^20): training steps/s
(events around K steps incl. Adam, after warm-up). The environment picks the variant under test
(e.g. TCNN_TILE_GENC=0 for the separate AoS encode pass)."""
import json, os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]
import torch
from bench import rgb_field_torch
from tinycudann import Trainer
cfg = json.load(open(os.path.join(REPO, "tests", "golden", "config_hash.json")))
cfg["network"] = {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": 128, "n_hidden_layers": 4}
B = 1 << int(os.environ.get("LOG2B", "20"))
K = int(os.environ.get("STEPS", "60"))
t = Trainer(2, 3, cfg, seed=1337)
g = torch.Generator(device="cuda"); g.manual_seed(1337)
batches = []
for _ in range(4):
    p = torch.rand(B, 2, device="cuda", generator=g)
    batches.append((p, rgb_field_torch(p)))
for i in range(10):
    t.training_step(*batches[i % 4])
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for i in range(K):
    t.training_step(*batches[i % 4])
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b) / K
print(json.dumps({"workload": "configs[3] HashGrid+W128/H4 B=2^%d" % B.bit_length() if False else f"configs[3] HashGrid+W128/H4 B={B}",
                  "genc": os.environ.get("TCNN_TILE_GENC", "default"), "ms_per_step": ms, "steps_per_s": 1000.0 / ms,
                  "loss": t.loss(), "engine": t.engine}))
