"""Diagnostic: tile-engine gradients per parameter block vs the oracle (NaN counts, rel errors)."""
import copy, json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd"), os.path.join(REPO, "tests")]
import numpy as np
import torch
from helpers import CONFIG_ONEBLOB, make_batch, trainer_arrays
from oracle import oracle as O
from tinycudann import Trainer
cfg = copy.deepcopy(CONFIG_ONEBLOB)
cfg["encoding"] = {"otype": "OneBlob", "n_bins": 16}
cfg["network"] = {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": 64, "n_hidden_layers": 2}
t = Trainer(2, 3, cfg, seed=1337)
print("engine", t.engine)
om = O.OracleModel(cfg, 2, 3, seed=1337)
pos, tgt = make_batch(512)
t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=False)
print("loss", t.loss(), om.train_step(pos, tgt, run_optimizer=False))
g = trainer_arrays(t)["g32"]
r = om.grad32
W, IN, NH = 64, 32, 2
blocks = [("W0", W * IN, IN)] + [(f"W{j}", W * W, W) for j in range(1, NH)] + [("Wout", 16 * W, W)]
o = 0
for name, n, cols in blocks:
    a, b = g[o:o + n].reshape(-1, cols), r[o:o + n].reshape(-1, cols)
    nan = np.isnan(a)
    print(name, "nan", nan.sum(), "of", n, "nan rows", sorted(set(np.nonzero(nan)[0].tolist()))[:20], "nan cols", sorted(set(np.nonzero(nan)[1].tolist()))[:20])
    ok = ~nan
    if ok.any():
        print("   rel err (finite)", np.linalg.norm(a[ok] - b[ok]) / max(np.linalg.norm(b[ok]), 1e-30), "max|ref|", np.abs(b).max(), "max|got|", np.nanmax(np.abs(a)))
    o += n
