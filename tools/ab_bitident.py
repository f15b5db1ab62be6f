# Bit-identity check between two builds of the engine (TCNN_LIB_PATH selects the library): a few
# training steps of config_hash at several batch sizes and position mixes; prints one digest per case
# (params fp32 + fp16 after 4 steps) and the 4 losses. Run once per build and compare the lines.
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd"))

import torch  # noqa: E402

from tinycudann import Trainer  # noqa: E402

cfg = json.load(open(os.path.join(REPO, "tests", "golden", "config_hash.json")))
g = torch.Generator(device="cuda").manual_seed(7)
for B, frac_out in ((1 << 15, 0.0), (1 << 18, 0.0), ((1 << 16) + 256, 0.0), (1 << 16, 0.002)):
    t = Trainer(2, 3, cfg, seed=1337)
    assert t.engine == "fused", t.engine
    h = hashlib.sha256()
    losses = []
    for step in range(4):
        pos = torch.rand(B, 2, device="cuda", generator=g)
        if frac_out:
            m = torch.rand(B, device="cuda", generator=g) < frac_out
            pos[m, 0] = 1.25
        tgt = torch.stack([0.5 + 0.5 * torch.sin(9 * pos[:, 0]), pos[:, 1], pos[:, 0] * pos[:, 1]], 1).contiguous()
        t.training_step(pos, tgt, run_optimizer=True)
        losses.append(t.loss())
    torch.cuda.synchronize()
    h.update(t.params_fp32().cpu().numpy().tobytes())
    h.update(t.params().cpu().numpy().tobytes())
    print("case", B, frac_out, h.hexdigest()[:16], "losses", " ".join("%.9g" % v for v in losses), flush=True)
    del t
