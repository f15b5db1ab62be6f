"""Diagnostic: run the fused training step a few times (for PMC passes)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd"), os.path.join(REPO, "tests")]
import torch
from helpers import CONFIG_HASH
from tinycudann import Trainer
B = 1 << 18
t = Trainer(2, 3, CONFIG_HASH)
pos = torch.rand(B, 2, device="cuda"); tgt = torch.rand(B, 3, device="cuda")
for _ in range(5):
    t.training_step(pos, tgt)
torch.cuda.synchronize()
print("ok")
