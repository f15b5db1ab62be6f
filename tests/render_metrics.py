"""Image helpers for the render pin (tests/test_render_pin.py, tests/test_gpu_render_pin.py,
tools/make_albert_full.py): binary PNM I/O, the 8-bit luma conversion and PSNR.

The reference's README shows the sample's renders after 100 and 1000 training steps of
data/config_hash.json on data/images/albert.jpg (README.md:69-79, data/readme/{100,1000}.jpg). They
are the only outputs of the reference's hot path anywhere in its tree. Their PSNR against the
training image (both decoded with the reference's own stb_image, oracle/_ref/stbi_decode) is frozen
in tests/golden/reference_renders.json; our engine's renders of the same run are scored with the
same function here."""
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ALBERT_FULL = os.path.join(GOLD, "albert_full.png")
REFERENCE_RENDERS = os.path.join(GOLD, "reference_renders.json")


def read_pnm(path):
    """binary PGM (P5) -> [H, W] uint8, PPM (P6) -> [H, W, 3] uint8"""
    with open(path, "rb") as f:
        data = f.read()
    magic, dims, maxval, body = data.split(b"\n", 3)
    w, h = map(int, dims.split())
    assert int(maxval) == 255, path
    if magic == b"P5":
        return np.frombuffer(body, np.uint8, count=w * h).reshape(h, w)
    assert magic == b"P6", path
    return np.frombuffer(body, np.uint8, count=w * h * 3).reshape(h, w, 3)


def write_pgm(path, img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    with open(path, "wb") as f:
        f.write(b"P5\n%d %d\n255\n" % (img.shape[1], img.shape[0]))
        f.write(img.tobytes())


def load_albert_full():
    """the training image, 4333 x 3250 8-bit gray (stb_image decode of albert.jpg)"""
    from PIL import Image  # PNG decode only (lossless)
    img = np.asarray(Image.open(ALBERT_FULL))
    assert img.shape == (4333, 3250) and img.dtype == np.uint8, img.shape
    return img


def luma(rgb):
    """ITU-R 601 8-bit luma, integer form (R 19595 + G 38470 + B 7471 + 2^15) >> 16"""
    if rgb.ndim == 2:
        return rgb
    r, g, b = (rgb[..., i].astype(np.uint32) for i in range(3))
    return ((r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16).astype(np.uint8)


def psnr(a, b):
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    mse = np.mean((a - b) ** 2)
    return float("inf") if mse == 0 else float(10.0 * np.log10(255.0 ** 2 / mse))


def psnr_gray(render, target):
    """PSNR of a render's luma against the gray training image"""
    return psnr(luma(render), target)


def linearise(img_u8):
    """stbi_loadf's 8-bit -> float conversion, pow(v / 255, 2.2) (stb_image.h:1838-1849)"""
    return np.power(img_u8.astype(np.float32) / np.float32(255.0), np.float32(2.2)).astype(np.float32)


def texture_targets(lin, pos):
    """the sample's training targets (eval_image, samples/mlp_learning_an_image.cu:83-99): the
    image's bilinear texture fetch at normalized coordinates with clamp addressing and 8-bit
    fractional weights, as the sample program computes it (mlp_learning_an_image.hip,
    sample_bilinear), in float32. lin: [H, W] linearised gray image; pos [B, 2] -> [B, 3]"""
    H, W = lin.shape
    f32 = np.float32
    x = pos[:, 0].astype(f32) * f32(W) - f32(0.5)
    y = pos[:, 1].astype(f32) * f32(H) - f32(0.5)
    fx, fy = np.floor(x), np.floor(y)
    ax = (np.rint((x - fx) * f32(256.0)) * f32(1.0 / 256.0)).astype(f32)
    ay = (np.rint((y - fy) * f32(256.0)) * f32(1.0 / 256.0)).astype(f32)
    x0 = np.clip(fx.astype(np.int64), 0, W - 1)
    x1 = np.clip(fx.astype(np.int64) + 1, 0, W - 1)
    y0 = np.clip(fy.astype(np.int64), 0, H - 1)
    y1 = np.clip(fy.astype(np.int64) + 1, 0, H - 1)
    one = f32(1.0)
    v = ((one - ax) * (one - ay) * lin[y0, x0] + ax * (one - ay) * lin[y0, x1] + (one - ax) * ay * lin[y1, x0] +
         ax * ay * lin[y1, x1]).astype(f32)
    return np.repeat(v[:, None], 3, axis=1)


def pixel_centres(H, W):
    """the sample's render coordinates ((x + 0.5) / W, (y + 0.5) / H), row-major [H * W, 2]"""
    xs = ((np.arange(W, dtype=np.float64) + 0.5) / W).astype(np.float32)
    ys = ((np.arange(H, dtype=np.float64) + 0.5) / H).astype(np.float32)
    out = np.empty((H, W, 2), dtype=np.float32)
    out[..., 0] = xs[None, :]
    out[..., 1] = ys[:, None]
    return out.reshape(-1, 2)


def to_ldr(v):
    """the sample's to_ldr (mlp_learning_an_image.cu:61-71): (uint8)(clamp(v)^(1/2.2) * 255 + 0.5)"""
    v = np.clip(v.astype(np.float32), 0.0, 1.0)
    return (np.power(v, np.float32(1.0 / 2.2)) * np.float32(255.0) + np.float32(0.5)).astype(np.uint8)


def load_reference_crops():
    """the reference's renders data/readme/{100,1000}.jpg, luma of a central crop
    (tests/golden/reference_render_crops.npz, tools/make_reference_render_crops.py)"""
    z = np.load(os.path.join(GOLD, "reference_render_crops.npz"))
    return {"100": z["render_100"], "1000": z["render_1000"],
            "rows": slice(int(z["crop_rows"][0]), int(z["crop_rows"][1])),
            "cols": slice(int(z["crop_cols"][0]), int(z["crop_cols"][1]))}


def render_vs_reference(render, img, crops, step):
    """render-to-render agreement with the reference's render of `step` on the fixture's crop: PSNR
    between the two renders and the correlation of their residuals against the training image"""
    ours = luma(render)[crops["rows"], crops["cols"]].astype(np.float64)
    ref = crops[step].astype(np.float64)
    a = img[crops["rows"], crops["cols"]].astype(np.float64)
    return {"psnr": psnr(ours, ref), "residual_corr": float(np.corrcoef((ours - a).ravel(), (ref - a).ravel())[0, 1])}
