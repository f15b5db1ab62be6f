import sys, os
sys.path[:0] = ['tests', '.', 'neuralbtf-tiny-cuda-nn_amd']
import numpy as np, torch
from helpers import CONFIG_HASH, make_batch, trainer_arrays
from oracle import oracle as O
from tinycudann import Trainer
t = Trainer(2, 3, CONFIG_HASH, seed=1337)
om = O.OracleModel(CONFIG_HASH, 2, 3, seed=1337)
for step in range(3):
    pos, tgt = make_batch(4096, step=step)
    before = trainer_arrays(t)
    t.training_step(torch.from_numpy(pos).cuda(), torch.from_numpy(tgt).cuda(), run_optimizer=True)
    a = trainer_arrays(t)
    m1, m2, st = [x.cpu().numpy().copy() for x in t.optimizer_state()]
    if step == 0:
        w32, w16 = before["w32"].copy(), before["w16"].copy()
        M1 = np.zeros_like(w32); M2 = np.zeros_like(w32); S = np.zeros(w32.size, np.uint32)
    O.adam_step(om.m.adam, om.n_mlp_params, 128.0, step + 1, w32, w16, a["g16"], M1, M2, S)
    d = np.nonzero(a["w32"] != w32)[0]
    print("step", step, "w32 mismatches", d.size, "m1", int(np.sum(m1 != M1)), "m2", int(np.sum(m2 != M2)), "steps", int(np.sum(st != S)))
    for i in d[:5]:
        print(i, a["w32"][i], w32[i], "m1", m1[i], M1[i], "m2", m2[i], M2[i], "g16", a["g16"][i])
    # continue from the GPU state to isolate one step at a time
    w32, w16, M1, M2, S = a["w32"].copy(), a["w16"].copy(), m1.copy(), m2.copy(), st.copy()
