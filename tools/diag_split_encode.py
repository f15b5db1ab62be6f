"""A/B of the fused training step's encoding (run under rocprofv3 --kernel-trace --stats, or alone for
wall-clock): config_hash.json at B = 2^18, (a) the fused kernel gathering the grid encoding in
registers (the default), (b) TCNN_SPLIT_ENCODE=1: the standalone SoA grid forward writes the encoding
and the fused kernel reads it (ENC_MEM). Also the Module forward (keep) + backward at the same batch.

  python tools/diag_split_encode.py
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]


def main():
    import torch
    from bench import rgb_field_torch
    from tinycudann import Trainer
    cfg = json.load(open(os.path.join(REPO, "tests", "golden", "config_hash.json")))
    B = 1 << 18
    pos = torch.rand(B, 2, device="cuda")
    tgt = rgb_field_torch(pos)
    res = {}
    for name, split in (("gather", False), ("split", True), ("gather2", False)):
        if split:
            os.environ["TCNN_SPLIT_ENCODE"] = "1"
        else:
            os.environ.pop("TCNN_SPLIT_ENCODE", None)
        t = Trainer(2, 3, cfg, seed=1337)
        for _ in range(20):
            t.training_step(pos, tgt)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            t.training_step(pos, tgt)
        torch.cuda.synchronize()
        res[name] = (time.perf_counter() - t0) / 200 * 1e6
        res[name + "_loss"] = t.loss()
        del t
    print(json.dumps({k: v for k, v in res.items()}))


if __name__ == "__main__":
    main()
