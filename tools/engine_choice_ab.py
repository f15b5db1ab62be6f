"""A/B of the engine choice for grid-encoded FullyFusedMLP shapes the register-resident fused kernel
takes (fused.hip TCNN_FUSED_SHAPES) against the tile engine (TCNN_NO_FUSED_GRID=1), HashGrid of
config_hash.json at B = 2^18, training steps incl. Adam. Each variant in its own child process.

  python tools/engine_choice_ab.py [--out profiles/r03_engine_choice_ab.json]
"""
import argparse
import copy
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd")]
SHAPES = [(64, 2), (64, 1), (64, 3), (32, 2), (32, 1)]


def child(iters):
    import torch
    from bench import rgb_field_torch
    from tinycudann import Trainer
    base = json.load(open(os.path.join(REPO, "tests", "golden", "config_hash.json")))
    B = 1 << 18
    pos = torch.rand(B, 2, device="cuda")
    tgt = rgb_field_torch(pos)
    rows = []
    for w, nh in SHAPES:
        cfg = copy.deepcopy(base)
        cfg["network"]["n_neurons"], cfg["network"]["n_hidden_layers"] = w, nh
        t = Trainer(2, 3, cfg, seed=1337)
        for _ in range(10):
            t.training_step(pos, tgt)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            t.training_step(pos, tgt)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / iters
        rows.append({"shape": f"W{w}/H{nh}", "ms_per_step": ms, "steps_per_s": 1000.0 / ms, "loss": t.loss()})
        del t
    print("ROWS " + json.dumps(rows), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        child(args.iters)
        return
    res = {}
    for v in ("fused", "tile"):
        env = dict(os.environ)
        env.pop("TCNN_NO_FUSED_GRID", None)
        if v == "tile":
            env["TCNN_NO_FUSED_GRID"] = "1"
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--iters", str(args.iters)], env=env,
                           capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-2000:]
        res[v] = json.loads([l for l in p.stdout.splitlines() if l.startswith("ROWS ")][0][5:])
    rows = [{"shape": f["shape"], "fused_kernel": f, "tile_engine": t, "tile_over_fused": f["ms_per_step"] / t["ms_per_step"]}
            for f, t in zip(res["fused"], res["tile"])]
    for r in rows:
        print(json.dumps(r), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"what": __doc__.split("\n\n")[0], "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
