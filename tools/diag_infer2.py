import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]
import torch
from helpers import CONFIG_HASH, make_batch
from oracle import oracle as O
from tinycudann import Trainer
om = O.OracleModel(CONFIG_HASH, 2, 3, seed=1337)
for B in (2048, 4096, 256):
    pos, _ = make_batch(B, seed=3)
    ref = O.h2f(om.inference(pos))[:, :3]
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    out = t.inference(torch.from_numpy(pos).cuda()).cpu().numpy()
    bad = ~np.isclose(out, ref, rtol=2e-3, atol=2e-4)
    rows = np.flatnonzero(bad.any(1))
    print("poisoned fresh B", B, "bad", bad.sum(), rows[:4], rows[-4:], "nan", np.isnan(out).sum(), flush=True)
