"""Seed-to-seed spread of the README experiment's render PSNR on the GPU (runs on the GPU box).

Runs the sample program (template API, config_hash.json, B = 2^18, full-resolution albert) for 1001
steps once per (batch seed, trainer seed) pair -- TCNN_SAMPLE_SEED / TCNN_SAMPLE_TRAINER_SEED -- and
scores the renders written after steps 0..10, 0..100 and 0..1000 like the reference's README images
(tests/render_metrics.py). The pair (1337, 1337) is the reference's own run. The spread sets the band
of tests/test_gpu_render_pin.py; the output is committed as tests/golden/render_spread.json.

Since r04 the reference's renders are known to come from batches of 2^16 points (tools/render_crops.py,
tools/render_compare.py); `16` as the second argument runs that batch (TCNN_SAMPLE_LOG2_BATCH) and
also scores each run's render crop against the reference's (tests/golden/reference_render_crops.npz:
render-to-render PSNR and residual correlation), which shows how far a different seed pair -- a
different run of the same pipeline -- lands from the reference's run.

usage: python tools/render_spread.py [out.json] [log2_batch]
"""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import render_metrics as RM  # noqa: E402

BIN = os.path.join(REPO, "neuralbtf-tiny-cuda-nn_amd", "bin", "mlp_learning_an_image")
SEEDS = [(1337, 1337), (1, 1337), (2, 1337), (3, 1337), (1337, 1), (1337, 2), (4, 4), (5, 5)]
STEPS = ("10", "100", "1000")


def run(img, seed, tseed, tmp, pgm, log2_batch=None, crops=None):
    env = dict(os.environ, TCNN_SAMPLE_SEED=str(seed), TCNN_SAMPLE_TRAINER_SEED=str(tseed))
    if log2_batch:
        env["TCNN_SAMPLE_LOG2_BATCH"] = str(log2_batch)
    t = time.time()
    out = subprocess.run([BIN, pgm, os.path.join(RM.GOLD, "config_hash.json"), "1001"], capture_output=True, text=True,
                         timeout=300, cwd=tmp, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    res = {"batch_seed": seed, "trainer_seed": tseed, "seconds": time.time() - t}
    for s in STEPS:
        p = os.path.join(tmp, f"{s}.ppm")
        r = RM.read_pnm(p)
        res[s] = RM.psnr_gray(r, img)
        if crops is not None and s in ("100", "1000"):
            res["vs_reference_render_" + s] = RM.render_vs_reference(r, img, crops, s)
        os.remove(p)
    return res


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "render_spread.json")
    log2_batch = int(sys.argv[2]) if len(sys.argv) > 2 else None
    crops = RM.load_reference_crops() if log2_batch else None
    img = RM.load_albert_full()
    runs = []
    with tempfile.TemporaryDirectory() as tmp:
        pgm = os.path.join(tmp, "albert.pgm")
        RM.write_pgm(pgm, img)
        for seed, tseed in SEEDS:
            runs.append(run(img, seed, tseed, tmp, pgm, log2_batch, crops))
            print(json.dumps(runs[-1]), flush=True)
    stats = {s: {"mean": float(np.mean([r[s] for r in runs])), "std": float(np.std([r[s] for r in runs], ddof=1)),
                 "min": float(np.min([r[s] for r in runs])), "max": float(np.max([r[s] for r in runs]))} for s in STEPS}
    res = {"what": "render PSNR (dB, gray) of the sample on config_hash.json, full-res albert, per seed pair"
                   + (f", batch 2^{log2_batch}" if log2_batch else ""),
           "log2_batch": log2_batch or 18, "runs": runs, "stats": stats}
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(stats, indent=1))


if __name__ == "__main__":
    main()
