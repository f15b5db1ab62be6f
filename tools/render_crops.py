"""Render crops of the README experiment per pipeline variant, for a render-to-render comparison with
the reference's own renders (runs on the GPU box; tools/render_compare.py scores them in the build
container, where the reference's data/readme/{100,1000}.jpg are).

PSNR against the training image measures how well a run learned; it cannot tell two pipelines of
equal quality apart. The reference's run and this sample share every seed (default_rng_t{1337}
batches, Trainer seed 1337, bit-exact pcg32 and initialisation), so a variant that reproduces the
reference's pipeline should reproduce its ERROR PATTERN (hash collisions, initial parameters, the
batches it saw) -- the render-vs-reference residuals then correlate far more than for a different
pipeline. Each variant writes the luma of a central crop of its 100- and 1000-step renders.

usage: python tools/render_crops.py [out_dir]
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import render_metrics as RM  # noqa: E402
from render_sweep import BIN, variants  # noqa: E402

CROP = (slice(1600, 2368), slice(1240, 2008))  # 768 x 768 around the face (rows, cols) of 4333 x 3250


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "render_crops")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(RM.GOLD, "config_hash.json")) as f:
        base = json.load(f)
    img = RM.load_albert_full()
    extra = [("batch=2^16+tex=exact", base, {"TCNN_SAMPLE_LOG2_BATCH": "16", "TCNN_SAMPLE_TEX_ROUND": "exact"}),
             ("batch=2^16+tex=trunc", base, {"TCNN_SAMPLE_LOG2_BATCH": "16", "TCNN_SAMPLE_TEX_ROUND": "trunc"})]
    with tempfile.TemporaryDirectory() as tmp:
        pgm = os.path.join(tmp, "albert.pgm")
        RM.write_pgm(pgm, img)
        np.save(os.path.join(out, "albert_crop.npy"), img[CROP])
        index = []
        for k, (name, cfg, env) in enumerate(variants(base) + extra):
            cfg_path = os.path.join(tmp, "config.json")
            with open(cfg_path, "w") as f:
                json.dump(cfg, f)
            e = dict(os.environ, **env)
            e.pop("TCNN_SAMPLE_SEED", None)
            e.pop("TCNN_SAMPLE_TRAINER_SEED", None)
            r = subprocess.run([BIN, pgm, cfg_path, "1001"], capture_output=True, text=True, timeout=300, cwd=tmp, env=e)
            assert r.returncode == 0, r.stdout + r.stderr
            for s in ("100", "1000"):
                np.save(os.path.join(out, f"v{k:02d}_{s}.npy"), RM.luma(RM.read_pnm(os.path.join(tmp, f"{s}.ppm")))[CROP])
            for s in ("0", "10", "100", "1000"):
                p = os.path.join(tmp, f"{s}.ppm")
                if os.path.exists(p):
                    os.remove(p)
            index.append({"k": k, "variant": name})
            print(k, name, flush=True)
    with open(os.path.join(out, "index.json"), "w") as f:
        json.dump({"crop_rows": [CROP[0].start, CROP[0].stop], "crop_cols": [CROP[1].start, CROP[1].stop],
                   "variants": index}, f, indent=1)


if __name__ == "__main__":
    main()
