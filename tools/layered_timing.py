"""Wall-clock ms/step of the layer-wise engine on BASELINE configs[1]/[3]-style models (diagnostic:
compare with the rocprofv3 kernel-time sum to see launch gaps)."""
import copy, json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "neuralbtf-tiny-cuda-nn_amd"))
import torch
from tinycudann import Trainer

GOLD = os.path.join(os.path.dirname(__file__), "..", "tests", "golden")
hashc = json.load(open(os.path.join(GOLD, "config_hash.json")))
oneb = json.load(open(os.path.join(GOLD, "config_oneblob.json")))
cases = {
    "oneblob_w128_h5_B2^18": (oneb, 1 << 18),
    "oneblob_w64_h2_B2^18": (dict(copy.deepcopy(oneb), network=dict(oneb["network"], n_neurons=64, n_hidden_layers=2)), 1 << 18),
    "hash_w128_h4_B2^20": (dict(copy.deepcopy(hashc), network=dict(hashc["network"], n_neurons=128, n_hidden_layers=4)), 1 << 20),
}
only = sys.argv[1] if len(sys.argv) > 1 else None
for name, (cfg, B) in cases.items():
    if only and only not in name:
        continue
    t = Trainer(2, 3, cfg)
    x = torch.rand(B, 2, device="cuda")
    y = torch.rand(B, 3, device="cuda")
    for _ in range(5):
        t.training_step(x, y)
    torch.cuda.synchronize()
    n = 30
    t0 = time.perf_counter()
    for _ in range(n):
        t.training_step(x, y)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / n
    print(json.dumps({"case": name, "engine": t.engine, "ms_per_step": round(ms, 4), "steps_per_s": round(1e3 / ms, 1)}), flush=True)
