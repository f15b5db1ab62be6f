"""Score tools/render_crops.py output against the reference's own renders (build container: needs
/root/reference/data/readme/{100,1000}.jpg and oracle/_ref/stbi_decode).

Per variant and step: PSNR of the variant's render crop against the reference render's crop, and the
correlation of the two renders' residuals against the training image (ours - albert vs
reference - albert). A variant with the reference's pipeline reproduces its error pattern: higher
render-to-render PSNR and residual correlation than any other variant.

usage: python tools/render_compare.py [crops_dir] [out.json]
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import render_metrics as RM  # noqa: E402

DEC = os.path.join(REPO, "oracle", "_ref", "stbi_decode")


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "render_crops")
    out_path = sys.argv[2] if len(sys.argv) > 2 else None
    idx = json.load(open(os.path.join(d, "index.json")))
    rows, cols = slice(*idx["crop_rows"]), slice(*idx["crop_cols"])
    albert = np.load(os.path.join(d, "albert_crop.npy")).astype(np.float64)
    ref = {}
    with tempfile.TemporaryDirectory() as tmp:
        for s in ("100", "1000"):
            o = os.path.join(tmp, s + ".ppm")
            subprocess.check_call([DEC, f"/root/reference/data/readme/{s}.jpg", o, "3"])
            ref[s] = RM.luma(RM.read_pnm(o))[rows, cols].astype(np.float64)
    res = []
    for v in idx["variants"]:
        row = {"variant": v["variant"]}
        for s in ("100", "1000"):
            ours = np.load(os.path.join(d, f"v{v['k']:02d}_{s}.npy")).astype(np.float64)
            ra, rb = (ours - albert).ravel(), (ref[s] - albert).ravel()
            row[s] = {"psnr_vs_reference_render": RM.psnr(ours, ref[s]), "psnr_vs_image": RM.psnr(ours, albert),
                      "residual_corr": float(np.corrcoef(ra, rb)[0, 1])}
        res.append(row)
        print(f"{v['variant']:22s} " + "  ".join(
            f"{s}: vs-ref {row[s]['psnr_vs_reference_render']:.2f} dB corr {row[s]['residual_corr']:.3f}" for s in ("100", "1000")))
    print("reference render vs image (crop): " + "  ".join(f"{s}: {RM.psnr(ref[s], albert):.2f} dB" for s in ("100", "1000")))
    if out_path:
        with open(out_path, "w") as f:
            json.dump({"what": "render-to-render comparison with data/readme/{100,1000}.jpg, crop rows/cols " +
                       str(idx["crop_rows"]) + str(idx["crop_cols"]), "variants": res}, f, indent=1)


if __name__ == "__main__":
    main()
