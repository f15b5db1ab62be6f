"""Inference workload for rocprofv3 --kernel-trace --stats: network->inference of data/config_oneblob.json
as-is (OneBlob 64 bins + FullyFusedMLP W128/H5) and BASELINE configs[3] (HashGrid + W128/H4) at
B = 2^18 and 2^21, 20 calls each (fused tile inference kernel k_mlp_tile_infer + the encoding pass).

  rocprofv3 --kernel-trace --stats -d out -o run -- python3 tools/prof_infer.py
"""
import copy
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]


def main():
    import torch
    from tinycudann import Trainer
    ob = json.load(open(os.path.join(REPO, "tests", "golden", "config_oneblob.json")))
    c3 = json.load(open(os.path.join(REPO, "tests", "golden", "config_hash.json")))
    c3 = copy.deepcopy(c3)
    c3["network"]["n_neurons"], c3["network"]["n_hidden_layers"] = 128, 4
    for name, cfg in (("config_oneblob", ob), ("configs3", c3)):
        t = Trainer(2, 3, cfg, seed=1337)
        assert t.inference_engine == "fused", t.inference_engine
        for lb in (18, 21):
            B = 1 << lb
            pos = torch.rand(B, 2, device="cuda")
            for _ in range(20):
                t.inference(pos)
            torch.cuda.synchronize()
            print(name, B, "ok", flush=True)
        del t


if __name__ == "__main__":
    main()
