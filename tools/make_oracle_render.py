"""The CPU oracle's run of the reference's README experiment (build container, a one-off of ~10 min):
config_hash.json on the full-resolution albert image, B = 2^18, batches from pcg32{1337} in
generate_random_uniform order, targets from the sample's bilinear texture fetch
(tests/render_metrics.py texture_targets), 101 training steps (the sample renders 100.jpg after steps
0..100), then the full 3250 x 4333 render and its PSNR against the training image.

Two modes, each stored under its own key of tests/golden/oracle_render.json (per-step losses and the
render PSNR):
  ideal  the oracle the GPU engine is checked against (fp32 accumulation, fp16 storage points);
  mimic  the reference-mimic rounding (oracle.set_mimic: fp16 WMMA / CUTLASS accumulators, fp16
         atomics into the grid gradient), i.e. the arithmetic of the reference's CUDA binary.
tests/test_render_pin.py re-runs the first steps on the live oracle (the losses must reproduce
exactly) and holds the PSNRs to the reference's own render (tests/golden/reference_renders.json).

The reference's renders were made with batches of 2^16 points (tools/render_crops.py +
tools/render_compare.py: that batch reproduces their error pattern, 42.5 dB render-to-render), so
`b16` runs the ideal-mode oracle at B = 2^16 under the key ideal_b16 (also saving a central crop of
its render, the one tools/render_crops.py takes, for the render-to-render check).

usage: python tools/make_oracle_render.py [ideal|mimic] [n_threads] [b16]
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import render_metrics as RM  # noqa: E402
from oracle import oracle as O  # noqa: E402

N_STEPS = 101
OUT = os.path.join(RM.GOLD, "oracle_render.json")


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "ideal"
    assert mode in ("ideal", "mimic"), mode
    nt = int(sys.argv[2]) if len(sys.argv) > 2 else os.cpu_count()
    b16 = len(sys.argv) > 3 and sys.argv[3] == "b16"
    B = 1 << (16 if b16 else 18)
    key = mode + ("_b16" if b16 else "")
    O.set_mimic(mode == "mimic")
    cfg = json.load(open(os.path.join(RM.GOLD, "config_hash.json")))
    img = RM.load_albert_full()
    lin = RM.linearise(img)
    om = O.OracleModel(cfg, 2, 3, seed=1337)
    rng = O.pcg32(1337)
    losses = []
    t0 = time.time()
    for i in range(N_STEPS):
        pos = O.generate_uniform(rng, 2 * B).reshape(B, 2)
        tgt = RM.texture_targets(lin, pos)
        losses.append(float(om.train_step(pos, tgt, run_optimizer=True, n_threads=nt)))
        print(f"step {i}: loss {losses[-1]:.6f} ({time.time() - t0:.0f} s)", flush=True)
    H, W = img.shape
    coords = RM.pixel_centres(H, W)
    n = coords.shape[0]
    npad = (n + 255) // 256 * 256
    render = np.empty((n, 3), dtype=np.uint8)
    CH = 1 << 20
    for s in range(0, npad, CH):
        e = min(s + CH, npad)
        c = np.zeros((e - s, 2), dtype=np.float32)
        m = min(e, n) - s
        c[:m] = coords[s:s + m]
        out = O.h2f(om.inference(c, n_threads=nt))[:m, :3]
        render[s:s + m] = RM.to_ldr(out)
        print(f"render {e}/{npad}", flush=True)
    render = render.reshape(H, W, 3)
    res = {
        "what": f"CPU oracle (oracle/tcnn_oracle.c, {mode} mode) running the reference README experiment: "
                f"config_hash.json, full-resolution albert, B = 2^{16 if b16 else 18}, pcg32{{1337}} batches, 8-bit-weight bilinear "
                "targets; render after steps 0..100",
        "batch": B,
        "losses": losses,
        "psnr_gray_100": RM.psnr_gray(render, img),
        "seconds": time.time() - t0,
        "threads": nt,
    }
    doc = json.load(open(OUT)) if os.path.exists(OUT) else {}
    if "losses" in doc:  # a single-run file from before the modes
        doc = {"ideal": doc}
    doc[key] = res
    if b16:
        from render_crops import CROP  # noqa: E402
        np.save(os.path.join(REPO, "gpurun_out", "oracle_b16_100_crop.npy"), RM.luma(render)[CROP])
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "losses"}, indent=1))


if __name__ == "__main__":
    main()
