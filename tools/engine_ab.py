"""A/B timing of the tile engine (mlp_tile.hip) against the layer-wise engine (TCNN_NO_TILE_ENGINE=1)
on the BASELINE configs it takes: configs[3] (HashGrid + W128/H4, B=2^20), configs[1] (OneBlob 64
bins + W64/H2, B=2^18), config_oneblob with W64 (H5), the sample's default (OneBlob 32 bins, W64/H4),
config_oneblob as-is (W128/H5, IN 128) and HashGrid + W128/H5 (hidden matrices streamed from L2).
Training steps (forward, loss, backward, Adam) timed with torch.cuda events after warm-up.

  python tools/engine_ab.py [--out profiles/r02_engine_ab.json]
"""
import argparse
import copy
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
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
    c = copy.deepcopy(ob); c["network"] = net(64, 2); cases.append(("configs[1] OneBlob64+W64/H2", c, 18))
    c = copy.deepcopy(ob); c["network"] = net(64, 5); cases.append(("config_oneblob W64/H5", c, 18))
    c = copy.deepcopy(ob); c["encoding"] = {"otype": "OneBlob", "n_bins": 32}; c["network"] = net(64, 4)
    cases.append(("sample default OneBlob32+W64/H4", c, 18))
    # shapes whose weights exceed the LDS: hidden matrices 1..NS streamed from L2 (mlp_tile.hip)
    cases.append(("config_oneblob as-is OneBlob64+W128/H5 (IN 128, 2 streamed)", copy.deepcopy(ob), 18))
    c = copy.deepcopy(hash_cfg); c["network"] = net(128, 5); cases.append(("HashGrid+W128/H5 (2 streamed)", c, 20))
    if os.environ.get("AB_ONLY_STREAMED"):
        cases = cases[-2:]
    rows = []
    for name, cfg, lb in cases:
        B = 1 << lb
        pos = torch.rand(B, 2, device="cuda")
        tgt = rgb_field_torch(pos)
        row = {"case": name, "batch": B}
        for eng, env in (("tile", None), ("layered", "1")):
            if env:
                os.environ["TCNN_NO_TILE_ENGINE"] = env
            else:
                os.environ.pop("TCNN_NO_TILE_ENGINE", None)
            t = Trainer(2, 3, cfg, seed=1337)
            for _ in range(5):
                t.training_step(pos, tgt)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.iters):
                t.training_step(pos, tgt)
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / args.iters
            row[eng] = {"engine": t.engine, "ms_per_step": ms, "steps_per_s": 1000.0 / ms, "loss": t.loss()}
            del t
        os.environ.pop("TCNN_NO_TILE_ENGINE", None)
        row["speedup"] = row["layered"]["ms_per_step"] / row["tile"]["ms_per_step"]
        rows.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(0), "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
