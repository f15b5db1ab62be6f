"""A/B timing of the tile engine's register-resident training variant (mlp_tile.h, tile_ra_ok: hidden
matrices' A fragments held in registers for the whole launch) against the LDS-staged one, on the tile
engine's BASELINE configs: configs[3] (HashGrid + W128/H4, B=2^20), configs[1] (OneBlob 64 bins +
W64/H2, B=2^18), the sample's default (OneBlob 32 + W64/H4) and config_oneblob with W64 (H5). Each
variant runs in its own child process (TCNN_TILE_REG_A is read once per process); training steps
timed with torch.cuda events after warm-up.

  python tools/tile_ra_ab.py [--out profiles/r03_tile_ra_ab.json]
"""
import argparse
import copy
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]


def cases():
    gold = os.path.join(REPO, "tests", "golden")
    hash_cfg = json.load(open(os.path.join(gold, "config_hash.json")))
    ob = json.load(open(os.path.join(gold, "config_oneblob.json")))

    def net(w, nh):
        return {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": w, "n_hidden_layers": nh}

    out = []
    c = copy.deepcopy(hash_cfg); c["network"] = net(128, 4); out.append(("configs[3] HashGrid+W128/H4", c, 20))
    c = copy.deepcopy(hash_cfg); c["network"] = net(128, 3); out.append(("HashGrid+W128/H3", c, 20))
    c = copy.deepcopy(ob); c["network"] = net(64, 2); out.append(("configs[1] OneBlob64+W64/H2", c, 18))
    c = copy.deepcopy(ob); c["encoding"] = {"otype": "OneBlob", "n_bins": 32}; c["network"] = net(64, 4)
    out.append(("sample default OneBlob32+W64/H4", c, 18))
    c = copy.deepcopy(ob); c["network"] = net(64, 5); out.append(("config_oneblob W64/H5", c, 18))
    return out


def child(iters):
    import torch
    from bench import rgb_field_torch
    from tinycudann import Trainer
    rows = []
    for name, cfg, lb in cases():
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
        rows.append({"case": name, "batch": B, "engine": t.engine, "ms_per_step": ms, "steps_per_s": 1000.0 / ms, "loss": t.loss()})
        del t
    print("ROWS " + json.dumps(rows), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        child(args.iters)
        return
    res = {}
    for v in ("0", "1"):
        env = dict(os.environ, TCNN_TILE_REG_A=v)
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--iters", str(args.iters)], env=env,
                           capture_output=True, text=True, timeout=300)
        print(p.stderr[-2000:], file=sys.stderr)
        assert p.returncode == 0, p.returncode
        res[v] = json.loads([l for l in p.stdout.splitlines() if l.startswith("ROWS ")][0][5:])
    rows = []
    for r0, r1 in zip(res["0"], res["1"]):
        row = {"case": r0["case"], "batch": r0["batch"], "lds_staged": r0, "register_resident": r1,
               "speedup": r0["ms_per_step"] / r1["ms_per_step"]}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"what": "tile training: register-resident A fragments (TCNN_TILE_REG_A=1) vs LDS-staged (=0)", "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
