"""A/B of the W128 tile kernel's samples per tile (TCNN_TILE_SAMPLES=32 vs the 64-sample default,
mlp_tile.h tile_ts64_ok): training steps (forward, loss, backward, Adam) of the W128 shapes that the
8-wave LDS-staged kernel runs, timed with torch.cuda events after warm-up. The switch is read once per
process, so run this script once per setting:

  TCNN_TILE_SAMPLES=32 python tools/tile_ts_ab.py ; python tools/tile_ts_ab.py
"""
import copy
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]


def main():
    import torch
    from bench import rgb_field_torch
    from tinycudann import Trainer
    gold = os.path.join(REPO, "tests", "golden")
    hash_cfg = json.load(open(os.path.join(gold, "config_hash.json")))
    ob = json.load(open(os.path.join(gold, "config_oneblob.json")))

    def net(w, nh):
        return {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": w, "n_hidden_layers": nh}

    cases = []
    c = copy.deepcopy(hash_cfg); c["network"] = net(128, 4); cases.append(("configs[3] HashGrid+W128/H4", c, 20))
    c = copy.deepcopy(ob); c["network"] = net(128, 3); cases.append(("OneBlob64+W128/H3 (IN 128)", c, 18))
    c = copy.deepcopy(ob); c["network"] = net(128, 2); cases.append(("OneBlob64+W128/H2 (IN 128)", c, 18))
    c = copy.deepcopy(ob); c["encoding"] = {"otype": "OneBlob", "n_bins": 32}; c["network"] = net(128, 4)
    cases.append(("OneBlob32+W128/H4 (IN 64)", c, 18))
    # the other tile-engine configurations (W64, W128/H5: the TCNN_TILE_SAMPLES switch does not apply)
    c = copy.deepcopy(ob); c["network"] = net(64, 2); cases.append(("configs[1] OneBlob64+W64/H2", c, 18))
    c = copy.deepcopy(ob); c["encoding"] = {"otype": "OneBlob", "n_bins": 32}; c["network"] = net(64, 4)
    cases.append(("sample default OneBlob32+W64/H4", c, 18))
    cases.append(("config_oneblob as-is OneBlob64+W128/H5 (IN 128)", copy.deepcopy(ob), 18))
    # the W128 register-resident kernel (IN <= 32, <= 3 hidden layers)
    c = copy.deepcopy(hash_cfg); c["network"] = net(128, 3); cases.append(("HashGrid+W128/H3 (register-resident)", c, 20))
    c = copy.deepcopy(hash_cfg); c["network"] = net(128, 2); cases.append(("HashGrid+W128/H2 (register-resident)", c, 20))
    iters = int(os.environ.get("ITERS", "30"))
    ts = os.environ.get("TCNN_TILE_SAMPLES", "default")
    for name, cfg, lb in cases:
        B = 1 << lb
        pos = torch.rand(B, 2, device="cuda")
        tgt = rgb_field_torch(pos)
        t = Trainer(2, 3, cfg, seed=1337)
        for _ in range(5):
            t.training_step(pos, tgt)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            t.training_step(pos, tgt)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / iters
        print(json.dumps({"case": name, "batch": B, "tile_samples": ts, "engine": t.engine, "ms_per_step": ms,
                          "steps_per_s": 1000.0 / ms, "loss": t.loss()}), flush=True)
        del t


if __name__ == "__main__":
    main()
