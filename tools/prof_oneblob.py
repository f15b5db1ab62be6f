"""config_oneblob.json as-is (OneBlob 64 bins + W128/H5, IN 128, B=2^18) training steps, for
rocprofv3 kernel statistics.  python tools/prof_oneblob.py [n_hidden_layers] [log2_batch] [n_neurons]
(BASELINE configs[1]: 2 18 64)"""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]
import torch
from bench import rgb_field_torch
from tinycudann import Trainer
cfg = json.load(open(os.path.join(REPO, "tests", "golden", "config_oneblob.json")))
if len(sys.argv) > 1:
    cfg["network"]["n_hidden_layers"] = int(sys.argv[1])
B = 1 << (int(sys.argv[2]) if len(sys.argv) > 2 else 18)
if len(sys.argv) > 3:
    cfg["network"]["n_neurons"] = int(sys.argv[3])
t = Trainer(2, 3, cfg, seed=1337)
pos = torch.rand(B, 2, device="cuda")
tgt = rgb_field_torch(pos)
for _ in range(25):
    t.training_step(pos, tgt)
torch.cuda.synchronize()
print("loss", t.loss(), "engine", t.engine)
