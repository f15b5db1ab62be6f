"""Diagnostic: trainer inference vs oracle after another trainer trained in the same process."""
import gc, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]
import torch
from helpers import CONFIG_HASH, make_batch, trainer_arrays
from oracle import oracle as O
from tinycudann import Trainer
om = O.OracleModel(CONFIG_HASH, 2, 3, seed=1337)
pos, _ = make_batch(2048, seed=3)
ref = O.h2f(om.inference(pos))[:, :3]
def check(tag, t):
    out = t.inference(torch.from_numpy(pos).cuda()).cpu().numpy()
    bad = ~np.isclose(out, ref, rtol=2e-3, atol=2e-4)
    rows = np.flatnonzero(bad.any(1))
    print(tag, "bad", bad.sum(), "rows", rows[:4], rows[-4:], flush=True)
    return out
def train(B, opt):
    t = Trainer(2, 3, CONFIG_HASH, seed=1337)
    p, g = make_batch(B)
    t.training_step(torch.from_numpy(p).cuda(), torch.from_numpy(g).cuda(), run_optimizer=opt)
    trainer_arrays(t)
for B, opt in ((256, False), (4096, False), (4096, True)):
    train(B, opt)
    gc.collect()
    t1 = Trainer(2, 3, CONFIG_HASH, seed=1337)
    check(f"after train B={B} opt={opt}", t1)
    torch.cuda.synchronize()
    check(f"  again (synced)", t1)
    del t1
