"""configs[3] (HashGrid + W128/H4, B=2^20) training steps, for rocprofv3 kernel statistics."""
import copy, json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]
import torch
from bench import rgb_field_torch
from tinycudann import Trainer
cfg = json.load(open(os.path.join(REPO, "tests", "golden", "config_hash.json")))
cfg["network"] = {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": 128, "n_hidden_layers": 4}
if len(sys.argv) > 1:
    cfg["encoding"]["log2_hashmap_size"] = int(sys.argv[1])
B = 1 << 20
t = Trainer(2, 3, cfg, seed=1337)
pos = torch.rand(B, 2, device="cuda")
tgt = rgb_field_torch(pos)
for _ in range(int(os.environ.get("STEPS", "25"))):
    t.training_step(pos, tgt)
torch.cuda.synchronize()
print("loss", t.loss(), "engine", t.engine)
