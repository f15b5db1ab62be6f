"""Per-workgroup phase times of the LDS grid backward (TCNN_DEBUG_GRID_TIMES=1 prints them to
stderr for every launch): config_hash at B=2^18, a few training steps.

  TCNN_DEBUG_GRID_TIMES=1 python tools/diag_grid_times.py 2> grid_times.txt
"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]
import json
import torch
from bench import rgb_field_torch
from tinycudann import Trainer
cfg = json.load(open(os.path.join(REPO, "tests", "golden", "config_hash.json")))
t = Trainer(2, 3, cfg, seed=1337)
B = 1 << int(os.environ.get("LOG2B", "18"))
pos = torch.rand(B, 2, device="cuda")
tgt = rgb_field_torch(pos)
for _ in range(int(os.environ.get("STEPS", "4"))):
    t.training_step(pos, tgt)
torch.cuda.synchronize()
print("done", t.loss())
